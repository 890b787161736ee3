"""GPU: the kernel-timing hook bench.py uses for the roofline (qfec_set_timing_events ->
hipExtLaunchKernel start/stop events).  The events must bracket the call's kernels, the
outputs must not change, and clearing the hook must stop the recording."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _events(n):
    import bench
    return bench.DeviceEvents(n)


def test_timing_events_bracket_the_kernels(engine, oracle):
    import torch
    from quic_amd import _lib, fec
    L = _lib.load()
    k, m, bb, G = 32, 4, 1352, 4096
    rng = np.random.default_rng(1)
    data_h = rng.integers(0, 256, (G, k, bb), dtype=np.uint8)
    data = torch.from_numpy(data_h).cuda()
    parity = torch.zeros((G, m, bb), dtype=torch.uint8, device="cuda")
    ev = _events(4)
    try:
        assert L.qfec_set_timing_events(ev.ev[0], ev.ev[1]) == 0
        engine.encode(k, m, bb, data, parity)
        assert L.qfec_set_timing_events(ev.ev[2], ev.ev[3]) == 0
        engine.encode(k, m, bb, data, parity)
        assert L.qfec_set_timing_events(None, None) == 0
        torch.cuda.synchronize()
        t1, t2 = ev.elapsed_ms(0, 1), ev.elapsed_ms(2, 3)
        assert 0 < t1 < 100 and 0 < t2 < 100
        # the second call's kernels start after the first call's end
        assert ev.elapsed_ms(1, 2) >= 0
        assert fec.last_kernels()
        # after clearing, calls record nothing: the stop event keeps its old time
        engine.encode(k, m, bb, data, parity)
        torch.cuda.synchronize()
        assert ev.elapsed_ms(2, 3) == pytest.approx(t2)
    finally:
        L.qfec_set_timing_events(None, None)
        ev.close()
    exp, rc = oracle.encode_batch(k, m, bb, data_h[:64])
    assert np.array_equal(parity[:64].cpu().numpy(), exp)
