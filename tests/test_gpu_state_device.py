"""State export / import through device buffers (fs2_get_state / fs2_set_state
with FS2_DEVICE), larger than one 256 MiB staging chunk.

The maps move through a staging buffer chunk by chunk; every copy must be
ordered on the handle's stream (a device-to-device hipMemcpy may return before
it ends, and the next chunk's memset or import kernel could overtake it: the
export then read back zeros).  Checked against the host-buffer path, then a
re-import through device buffers followed by scans must equal a handle that was
never re-imported (reference: Particle.landmarks round trips,
fast_slam_2.py:20-31 / models/particle.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_device_state_roundtrip_chunks():
    import torch
    import fast_slam_2
    import fs2_synthetic as syn
    from fast_slam_2 import _native as nat
    from gpu_util import configure
    configure()
    N, L, cap = 30_000, 560, 600           # 256 MiB / (600 * 48 B) = 9320 particles per staging chunk
    wl = syn.Workload(N, L, seed=3)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    hs = [fast_slam_2.FastSLAM2(N, reduce="auto", rng="device", seed=4, landmark_capacity=cap, record_assoc=True,
                                verbose=False)
          for _ in range(2)]
    for h in hs:
        h.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
    for s in range(3):
        for h in hs:
            h.step(*syn.odometry(s), wl.measurements(s))
    host = hs[1].get_state(lm_cap=cap)
    f = hs[1]
    dl = torch.full((N, cap, 6), -7.0, dtype=torch.float64, device="cuda")
    dc = torch.zeros(N, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    nat.check(f._lib.fs2_get_state(f._h, 0, N, None, None, None, None, dc.data_ptr(), dl.data_ptr(), cap,
                                   nat.FS2_DEVICE), f._h)
    torch.cuda.synchronize()
    assert np.array_equal(dc.cpu().numpy(), host[4])
    live = np.arange(cap)[None, :] < host[4][:, None]
    assert np.array_equal(dl.cpu().numpy()[live], host[5][live])
    # re-import through the device buffers (fresh pages and records), then continue
    nat.check(f._lib.fs2_set_state(f._h, 0, N, None, None, None, None, dc.data_ptr(), dl.data_ptr(), cap,
                                   nat.FS2_DEVICE), f._h)
    again = f.get_state(lm_cap=cap)
    assert np.array_equal(again[4], host[4])
    assert np.array_equal(again[5][live], host[5][live])
    for s in range(3, 6):
        (p0, s0), (p1, s1) = [h.step(*syn.odometry(s), wl.measurements(s)) for h in hs]
        assert np.array_equal(p0, p1) and s0.resampled == s1.resampled, s
        assert np.array_equal(hs[0].associations(), hs[1].associations()), s
    a, b = hs[0].get_state(lm_cap=cap), hs[1].get_state(lm_cap=cap)
    for u, v in zip(a, b):
        assert np.array_equal(u, v)
    for h in hs:
        h.close()
