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
        err = buf[done_off + 8:done_off + 16].view(np.int64)
        err[0] = 0
        for n in range(7):
            k = n % n_slots
            words[k] = np.arange(slot_bytes // 4, dtype=np.uint32) + 1000 * (n + 1)
            words[k][-2:].view(np.int64)[0] = n         # the slot's replay tag
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
            assert int(err[0]) == 0
        # a slot written for another replay: flagged (sticky, the first mismatch's count + 1), copied anyway
        for n in (7, 8):
            k = n % n_slots
            words[k][-2:].view(np.int64)[0] = n + 3
            _lib.call("nerf_scalars_fetch", h.value, slot_bytes, n_slots, done_off, _lib.ptr(ctl, "ctl", torch.int64),
                      dst.data_ptr(), _lib.stream())
            torch.cuda.synchronize()
            assert int(err[0]) == 8 and int(done[0]) == n + 1
        with pytest.raises(RuntimeError):    # done word inside the slots
            _lib.call("nerf_scalars_fetch", h.value, slot_bytes, n_slots, 8, _lib.ptr(ctl, "ctl", torch.int64),
                      dst.data_ptr(), _lib.stream())
    finally:
        _lib.call("nerf_host_ring_free", h.value)


def test_step_scalars_detects_parted_counts(gpu):
    """graphs.StepScalars: a replay without its upload() fetches a slot written for an earlier replay
    (its tag is that replay's index, not the device count): the fetch flags it and the next upload()
    raises instead of training on another step's scalars. seal() re-synchronises. (An upload without
    its replay can only come from an exception between the two; GraphedTrainStep re-seals then.)"""
    from indoor_nerf_amd.graphs import StepScalars
    sc = StepScalars(gpu, n_i64=8, n_f32=8, ring=2)
    off, dptr = sc.alloc_i64(1)
    sc.add_filler(lambda hi, hf: hi.__setitem__(off, 100 + sc.issued))
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(device=gpu)
    with torch.cuda.stream(side), torch.cuda.graph(g, stream=side):
        sc.capture_fetch()
    torch.cuda.current_stream(gpu).wait_stream(side)
    sc.seal()
    for n in range(3):
        sc.upload()
        g.replay()
        torch.cuda.synchronize()
        assert int(sc.dev_i[off]) == 100 + n
    assert int(sc.err[0]) == 0
    g.replay()             # no upload: replay 3 fetches slot 1, written for replay 1
    torch.cuda.synchronize()
    assert int(sc.err[0]) == 4
    with pytest.raises(RuntimeError, match="parted"):
        sc.upload()
    sc.seal()
    sc.upload()
    g.replay()
    torch.cuda.synchronize()
    assert int(sc.dev_i[off]) == 100 and int(sc.err[0]) == 0
