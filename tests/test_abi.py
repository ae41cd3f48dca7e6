"""CPU-only checks of the C ABI library and the C oracle."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    txt = open(os.path.join(ROOT, "include", "nerf_hip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const char\*|int|int64_t|size_t)\s+(nerf_\w+)\s*\(", txt, flags=re.M)))


def test_library_exports_every_declared_symbol(nerf):
    import indoor_nerf_amd._lib as L
    lib = nerf.load_library()
    declared = _declared_symbols()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), f"libnerfhip.so does not export {name}"
    assert sorted(L.exported_symbols()) == declared, "ctypes signature table out of sync with the header"
    assert lib.nerf_abi_version() == 12   # 12: nerf_normal_head_fwd_rows; 11: TV bins in the hash bin launch (nerf_hash_encode_bwd_bin_batch_tv); 10: saved h3 (nerf_mlp_fwd_h3, job.h3); 9: RAdam grad_scale


def test_error_path_reports_message(nerf):
    """Argument validation runs on the host, without touching a GPU."""
    import indoor_nerf_amd._lib as L
    with pytest.raises(RuntimeError, match="n_levels"):
        L.call("nerf_hash_encode_fwd", None, 1, L.host_f32([0] * 3), L.host_f32([1] * 3), L.host_f32([16]), 0, 19,
               None, None, 2, 2, None, None)
    with pytest.raises(RuntimeError, match="S must be"):
        L.call("nerf_composite_fwd", None, 4, None, None, None, 4, 1000, 0, *([None] * 7), None)
    # split binned backward: the chunk range and the workspace size are checked before any launch
    C = L.load().nerf_hash_bwd_chunk_points()
    need = L.load().nerf_hash_encode_bwd_workspace_bytes(16, 19, C * 4, 0)
    fake = ctypes.c_void_p(1 << 20)
    with pytest.raises(RuntimeError, match="n_chunks 5 of 4"):
        L.call("nerf_hash_encode_bwd_owner", 16, 19, 5, 4, None, 0, fake, need, None)
    with pytest.raises(RuntimeError, match="workspace"):
        L.call("nerf_hash_encode_bwd_owner", 16, 19, 4, 4, None, 0, fake, need - 1, None)
    with pytest.raises(RuntimeError, match="flags 4"):   # bit 0 deterministic, bit 1 overwrite, nothing else
        L.call("nerf_hash_encode_bwd_owner", 16, 19, 4, 4, None, 4, fake, need, None)
    with pytest.raises(RuntimeError, match="exceed the capacity"):
        L.call("nerf_hash_encode_bwd_bin", fake, 3 * C + 1, L.host_f32([0] * 3), L.host_f32([1] * 3),
               L.host_f32([16] * 16), 16, 19, fake, 32, 2, 1, 4, 0, fake, need, None)
    # the deterministic plan is larger (2^12-row slices, per-level maxima): the plain size is refused
    need_det = L.load().nerf_hash_encode_bwd_workspace_bytes(16, 19, C * 4, 1)
    assert need_det > need
    with pytest.raises(RuntimeError, match="workspace"):
        L.call("nerf_hash_encode_bwd_owner", 16, 19, 4, 4, None, 1, fake, need, None)
    with pytest.raises(RuntimeError, match="deterministic"):
        L.call("nerf_hash_encode_bwd_ws", fake, 10, L.host_f32([0] * 3), L.host_f32([1] * 3), L.host_f32([16] * 16),
               16, 19, fake, 32, 2, (ctypes.c_void_p * 16)(*[1 << 20] * 16), 1, None, 0, None)
    # empty batches still validate the tables and host arrays
    with pytest.raises(RuntimeError, match="grad table 3 is null"):
        L.call("nerf_hash_encode_bwd_ws", None, 0, L.host_f32([0] * 3), L.host_f32([1] * 3), L.host_f32([16] * 16),
               16, 19, None, 32, 2, (ctypes.c_void_p * 16)(*([1 << 20] * 3 + [None] + [1 << 20] * 12)), 0, None, 0, None)
    with pytest.raises(RuntimeError, match="1..2"):
        L.call("nerf_mlp_bwd_batch", (L.MlpBwdJob * 3)(), 3, None, 0, None)


def test_empty_batches_accept_null_data(nerf):
    """Zero rays / points: the entries return NERF_OK before any launch and, like torch's empty
    tensors (data_ptr 0), accept NULL per-point buffers; the same NULLs with one point are refused.
    Host-only (no GPU call is reached)."""
    import indoor_nerf_amd._lib as L
    bb = (L.host_f32([0] * 3), L.host_f32([1] * 3), L.host_f32([16] * 16))
    tabs = (ctypes.c_void_p * 16)(*([1 << 20] * 16))
    for n, ok in ((0, True), (1, False)):
        calls = [
            lambda: L.call("nerf_sample_stratified", None, 11, n, 64, None, 0, 0, None, 0, 0, None, None, None, None,
                           None, None),
            lambda: L.call("nerf_composite_fwd", None, 4, None, None, None, n, 64, 0, *([None] * 7), None),
            lambda: L.call("nerf_hash_encode_fwd", None, n, *bb, 16, 19, tabs, None, 2, 2, None, None),
            lambda: L.call("nerf_hash_encode_bwd", None, n, *bb, 16, 19, None, 2, 2, tabs, None),
            lambda: L.call("nerf_sh4_fwd", None, n, None, None),
            # A-CAQ: eval-mode int-packed gather and the calibration's corner min/max
            lambda: L.call("nerf_hash_encode_fwd_packed", None, n, *bb, 16, 19, ctypes.c_void_p(1 << 20),
                           ctypes.c_void_p(1 << 20), None, 2, 2, None, None),
            lambda: L.call("nerf_hash_gather_minmax", None, n, *bb, 16, 19, tabs, ctypes.c_void_p(1 << 20), None),
        ]
        for c in calls:
            if ok:
                c()
            else:
                with pytest.raises(RuntimeError, match="null|bad args"):
                    c()


def test_mlp_refuses_batches_past_32bit_indexing(nerf):
    """The MLP kernels form 32-bit element indices: a batch whose feature / output indices would
    pass 2^31 is refused on the host before any launch (2^27 points x 16 levels), one below is not
    checked here (it would launch)."""
    import indoor_nerf_amd._lib as L
    fake = ctypes.c_void_p(1 << 20)
    w = L.MlpWeights(*([1 << 20] * 5))
    P = 1 << 27
    with pytest.raises(RuntimeError, match="32-bit indexing"):
        L.call("nerf_mlp_fwd", fake, 2, 2 * P, None, 0, fake, 192, None, P, ctypes.byref(w), fake, None, None)


def _oracle_lib():
    path = os.path.join(ROOT, "oracle", "_build", "libhashgrid_ref.so")
    if not os.path.exists(path):
        import __graft_entry__ as g
        g.build_oracle()
    lib = ctypes.CDLL(path)
    lib.hashgrid_ref_fwd.restype = None
    return lib


def _c_hash(xyz, res, table, want_idx=False):
    from tables import blender_bbox
    lib = _oracle_lib()
    lo, hi = blender_bbox()
    n, L = xyz.shape[0], len(res)
    feat = np.zeros((n, 2 * L), np.float32)
    keep = np.zeros(n, np.uint8)
    idx = np.zeros((n, L, 8), np.int32)
    vmin = np.zeros((n, L, 3), np.float32)
    vmax = np.zeros((n, L, 3), np.float32)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    xyz = np.ascontiguousarray(xyz, np.float32)
    lo, hi, res = (np.ascontiguousarray(v, np.float32) for v in (lo, hi, res))
    lib.hashgrid_ref_fwd(P(xyz), ctypes.c_int64(n), P(lo), P(hi), P(res), len(res), 19, P(table), P(feat), P(keep),
                         P(idx), P(vmin), P(vmax))
    return feat, keep.astype(bool), idx, vmin, vmax


def test_c_oracle_voxel_exact(golden):
    from tables import closed_form_table
    g = golden("f2_voxel")
    res = golden("f1_levels")["res_1024"]
    _, keep, idx, vmin, vmax = _c_hash(g["xyz"], res, closed_form_table())
    np.testing.assert_array_equal(idx, g["idx"])
    np.testing.assert_array_equal(vmin, g["vmin"])
    np.testing.assert_array_equal(vmax, g["vmax"])
    np.testing.assert_array_equal(keep, g["keep"])


def test_c_oracle_hash_fwd_exact(golden):
    from tables import closed_form_table
    g = golden("f3_hash_fwd")
    lv = golden("f1_levels")
    table = closed_form_table()
    for finest in (512, 1024):
        feat, keep, *_ = _c_hash(g[f"xyz_{finest}"], lv[f"res_{finest}"], table)
        np.testing.assert_array_equal(feat, g[f"feat_{finest}"])
        np.testing.assert_array_equal(keep, g[f"keep_{finest}"])


def test_hash_bwd_workspace_plan(nerf):
    """Host-side plan of the binned backward (csrc/hashgrid.hip make_bin_plan): per level and
    C-point chunk (C = nerf_hash_bwd_chunk_points()) a region of 8 C entries (8-B d feat + 2-B row) and n_owner segment words, each
    array 256-B aligned; owner slices of min(2^13, T) rows, at most 128 owners (log2_T <= 20)."""
    lib = nerf.load_library()
    C = lib.nerf_hash_bwd_chunk_points()
    assert C in (256, 512, 1024)
    up = lambda v: (v + 255) // 256 * 256  # noqa: E731
    for L, log2_T, P in ((16, 19, 786432), (16, 19, 262144), (8, 12, 1000), (16, 14, 5), (16, 20, 1000)):
        for det, slice_log2 in ((0, 13), (1, 12)):   # deterministic: 2^12-row slices + per-chunk maxima
            if det and log2_T > 19:
                assert lib.nerf_hash_encode_bwd_workspace_bytes(L, log2_T, P, det) == 0
                continue
            nch = (P + C - 1) // C
            own = 1 << (log2_T - min(slice_log2, log2_T))
            ent = L * nch * 8 * C
            expect = up(ent * 8) + up(ent * 2) + up(L * nch * own * 4) + (up(L * nch * 4) if det else 0)
            assert lib.nerf_hash_encode_bwd_workspace_bytes(L, log2_T, P, det) == expect
    assert lib.nerf_hash_encode_bwd_workspace_bytes(16, 21, 1000, 0) == 0
    assert lib.nerf_hash_encode_bwd_workspace_bytes(0, 19, 1000, 0) == 0


def test_tv_bin_chunks(nerf):
    """nerf_tv_bwd_bin_chunks: the chunks of the binned TV backward = max over levels of
    ceil((cube + 1)^3 / (8 C)) (8 vertices per thread of a C-thread bin block); 0 for bad input."""
    import indoor_nerf_amd._lib as L
    lib = nerf.load_library()
    C = lib.nerf_hash_bwd_chunk_points()
    cubes = [15] * 9 + [19, 25, 33, 44, 50, 50, 50]
    arr = (L.c_int * 16)(*cubes)
    assert lib.nerf_tv_bwd_bin_chunks(16, arr) == max(-(-(c + 1) ** 3 // (8 * C)) for c in cubes)
    assert lib.nerf_tv_bwd_bin_chunks(0, arr) == 0
    assert lib.nerf_tv_bwd_bin_chunks(1, (L.c_int * 1)(0)) == 0


def test_crop_window_matches_reference_grid(golden):
    """RaySampler's cell -> pixel map over the precrop window equals train()'s coords grid
    (run_nerf.py:985-996), F16 (precrop_frac 0.5 on a 60 x 80 image); full image after precrop."""
    from indoor_nerf_amd.rays import crop_window
    g = golden("f16_rays")
    H, W = int(g["H"]), int(g["W"])
    r0, c0, h, w = crop_window(H, W, 3, precrop_iters=500, precrop_frac=0.5)
    k = np.arange(h * w)
    np.testing.assert_array_equal(np.stack([r0 + k // w, c0 + k % w], -1), g["crop_coords"])
    assert crop_window(H, W, 500, precrop_iters=500) == (0, 0, H, W)
