"""nerf_scalars_fetch (graphs.StepScalars): each launch copies ring slot (count mod n_slots) into the
device slots, only the two word ranges the control block names, advances the device count and
publishes it in the ring's done word."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_fetch_cycles_the_ring(gpu):
    from indoor_nerf_amd import _lib
    slot_bytes, n_slots = 256, 3
    done_off = n_slots * slot_bytes
    h = ctypes.c_void_p()
    _lib.call("nerf_host_ring_alloc", done_off + 64, ctypes.byref(h))
    try:
        buf = np.ctypeslib.as_array((ctypes.c_uint8 * (done_off + 64)).from_address(h.value))
        words = buf[:done_off].view(np.uint32).reshape(n_slots, slot_bytes // 4)
        done = buf[done_off:done_off + 8].view(np.int64)
        done[0] = 0
        dst = torch.full((slot_bytes // 4,), 0xDEAD, dtype=torch.int32, device=gpu)
        ctl = torch.tensor([0, 5, 40, 3], dtype=torch.int64, device=gpu)   # words [0,5) and [40,43)
        for n in range(7):
            k = n % n_slots
            words[k] = np.arange(slot_bytes // 4, dtype=np.uint32) + 1000 * (n + 1)
            _lib.call("nerf_scalars_fetch", h.value, slot_bytes, n_slots, done_off, _lib.ptr(ctl, "ctl", torch.int64),
                      dst.data_ptr(), _lib.stream())
            torch.cuda.synchronize()
            got = dst.cpu().numpy().view(np.uint32)
            want = np.full(slot_bytes // 4, 0xDEAD, dtype=np.uint32)
            idx = np.r_[0:5, 40:43]
            want[idx] = words[k][idx]
            np.testing.assert_array_equal(got, want)
            assert int(ctl[0]) == n + 1 and int(done[0]) == n + 1
            assert int(ctl[1]) == 5 and int(ctl[2]) == 40 and int(ctl[3]) == 3
        with pytest.raises(RuntimeError):    # done word inside the slots
            _lib.call("nerf_scalars_fetch", h.value, slot_bytes, n_slots, 8, _lib.ptr(ctl, "ctl", torch.int64),
                      dst.data_ptr(), _lib.stream())
    finally:
        _lib.call("nerf_host_ring_free", h.value)
