"""Host restatement of the device scene generator (avz_scene_generate, csrc/avz_scene.hip):
Philox4x32-10 against Random123's published known-answer vectors, the draw streams'
statistics and independence, and mix_draws against make_scene (the reference-model mixer,
world_building.py:47-59 / simulation.py:167-202) on identical draws."""
import numpy as np

from avz import synth


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32 with 10 rounds: (ctr, key) -> out
    kat = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, want in kat:
        assert tuple(int(v) for v in synth.philox4x32(*ctr, *key)) == want


def test_normal_and_uniform_streams():
    key = synth._key(12345)
    z = synth.philox_normals(key, 0, 200000)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01
    assert abs(np.mean(z ** 4) - 3.0) < 0.05  # Gaussian kurtosis
    u = synth.philox_uniform(key, np.arange(100000))
    assert u.min() >= 0.0 and u.max() < 1.0 and abs(u.mean() - 0.5) < 0.01
    # streams and keys are independent; draws are a pure function of (key, stream, index)
    z1 = synth.philox_normals(key, 1, 200000)
    assert abs(np.corrcoef(z, z1)[0, 1]) < 0.01
    assert np.array_equal(synth.philox_normals(key, 0, 1000), z[:1000])
    assert not np.array_equal(synth.philox_normals(synth._key(12346), 0, 1000), z[:1000])
    assert not np.array_equal(synth.philox_normals(synth._key(12345, seed=1), 0, 1000), z[:1000])


def test_philox_scene_conventions():
    n = 16000
    a, s, z = synth.scene_draws_philox(9, n, 3)
    assert a[0] == 90.0 and a[1] == 40.0 and np.all((a[2:] >= 0) & (a[2:] < 180))
    assert s.shape == (4, n) and z.shape == (2, n)
    # 250-ms blocks are either silent or carry the |sin| envelope
    blk = s.reshape(4, -1, 4000)
    assert np.all((np.abs(blk).max(axis=2) == 0) | (np.abs(blk).max(axis=2) > 0.1))
    mix, tgt, itf = synth.make_scene_philox(9, n, 3)
    assert mix.dtype == np.float32 and abs(np.abs(mix).max() - 1.0) < 1e-6
    m2, _, _ = synth.make_scene_philox(9, n, 3)
    assert np.array_equal(mix, m2)


def test_mix_draws_restates_make_scene():
    """mix_draws on make_scene's own draws (scene_draws, same RNG order) gives make_scene."""
    for idx, k in ((5, 2), (11, 1), (3, 0)):
        a, s, z = synth.scene_draws(idx, 8000, k)
        got = synth.mix_draws(a, s, z)
        want = synth.make_scene(idx, 8000, k)
        for g, w in zip(got, want):
            np.testing.assert_allclose(g, w, rtol=0, atol=1e-7)
