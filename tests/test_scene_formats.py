"""Scene writers of the synthetic generator (avz/synth.py) against the reference's
formats: world_building.mix_and_save (full_audio_generating_pipeline/world_building.py:
68-100) pinned by a reference run (tests/golden/world_mix.npz), and the world.py /
Final_pipeline/src/simulation.py file layouts read back through avz.wavio. CPU only."""
import os

import numpy as np

from conftest import golden


def test_mix_and_save_matches_reference(tmp_path):
    from avz import synth
    g = golden("world_mix.npz")
    srcs = [(s.astype(np.float64) / 32768.0).astype(np.float32) for s in g["sources"]]
    mix, tgt, itf = synth.mix_and_save(srcs, "golden", angles=tuple(g["angles"]),
                                       d=float(g["d"]), out_dir=str(tmp_path))
    np.testing.assert_allclose(mix.T, g["mixture"], atol=1e-12)
    np.testing.assert_allclose(tgt, g["target_ref"], atol=1e-12)
    np.testing.assert_allclose(itf, g["interf_ref"], atol=1e-12)
    for f in ("mixture_golden.wav", "target_ref_golden.wav", "interf_ref_golden.wav"):
        assert os.path.exists(tmp_path / f)


def test_world_and_final_pipeline_layouts(tmp_path):
    from avz import synth, wavio
    mix, tgt, itf = synth.make_scene(3, n_samples=8000, n_interferers=2)
    d = synth.write_world_scene(str(tmp_path / "world"), mix, tgt, itf)
    m, fs = wavio.read(os.path.join(d, "mixture.wav"))
    t, _ = wavio.read(os.path.join(d, "target_reference.wav"))
    i, _ = wavio.read(os.path.join(d, "interference_reference.wav"))
    assert fs == 16000 and m.shape == (8000, 2) and t.shape == (8000,) and i.shape == (8000,)
    q = 1.0 / 32768
    assert np.max(np.abs(m - mix.T)) <= q
    # world.py:243-244: each reference peak-normalised on its own
    assert abs(np.max(np.abs(t)) - 1.0) <= 2 * q and abs(np.max(np.abs(i)) - 1.0) <= 2 * q
    p = synth.write_final_pipeline_scene(str(tmp_path / "fp"), mix, tgt, itf)
    tt, _ = wavio.read(os.path.join(os.path.dirname(p), "target.wav"))
    ii, _ = wavio.read(os.path.join(os.path.dirname(p), "interference.wav"))
    assert tt.shape == (8000, 2) and ii.shape == (8000, 2)
    # simulation.py:197-202: shared scale with the mixture
    assert np.max(np.abs(tt[:, 0] - tgt)) <= q and np.max(np.abs(ii[:, 0] - itf)) <= q
