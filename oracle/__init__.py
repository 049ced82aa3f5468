"""CPU oracle for the mask-driven MVDR hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker / the timed CPU baseline.
The product path (``avz``) never imports it and has no CPU fallback.

Parity status: PINNED. ``tests/test_oracle_golden.py`` checks this restatement
against golden vectors produced by running the reference itself in the build
container (``tests/golden/make_golden.py``; fixtures in ``tests/golden/``).
"""
