"""Phase timeline of the device priors' single-workgroup launches (csrc/priors_fused.hip), a
diagnostic: `--patch DIR` writes a copy of the kernel source into DIR with wall_clock64() stamps
(thread 0, 100 MHz) at the phase boundaries, stored over the workspace's `members` rows (unused in
device mode); `--run` (from inside DIR, after building it) runs the device path on a ScanNet-sized
batch and prints each phase's duration in us, averaged over repetitions."""
import os
import re
import sys

PHASES = [  # (kernel-relative anchor regex, stamp index, name); stamped right AFTER the matched line
    (r"PriorsState& st = \*a\.st;\n    const int N = a\.N, tid = threadIdx\.x;\n    int ns = 0, nf = 0, nw = 0, nk = 0;", 0, "prep: start"),
    (r"block_sum_vec<4>\(c4, s_red\);", 1, "prep: normals pass + counts"),
    (r"        for \(int c = 0; c < 3; \+\+c\) s_c\[3 \* tid \+ c\] = r\[c\] / d;\n    \}\n    __syncthreads\(\);", 2, "prep: k-means init"),
    (r"            a\.assign\[\(size_t\)it \* N \+ i\] = asg;\n        \}", 40, "round: points"),
    (r"        block_sum_vec<12>\(red, s_red\);\n        __syncthreads\(\);", 41, "round: 12 sums"),
    (r"                st\.centre_count\[k\] = \(int\)red\[9 \+ k\];\n            \}\n        \}\n        __syncthreads\(\);", 3, "prep: k-means round (each)"),
    (r"    if \(tid < 9\) st\.centres\[tid\] = s_c\[tid\];", 13, "prep: end"),
    (r"s_keys\[\];[^\n]*\n    PriorsState& st = \*a\.st;\n    const int N = a\.N, tid = threadIdx\.x;\n"
     r"    const float scale = a\.d_scale \? \*a\.d_scale : 1\.0f;", 16, "loss: start"),
    (r"        st\.flip = flip;\n    \}\n    __syncthreads\(\);", 17, "loss: frame"),
    (r"block_sum_vec<4>\(r4, s_red\);", 18, "loss: manhattan"),
    (r"            s_keys\[i\] = key;\n        \}", 19, "loss: sort keys"),
    (r"        bitonic_sort\(s_keys, M2\);", 20, "loss: bitonic sort"),
    (r"block_sum_vec<3>\(part, s_red\);", 22, "loss: pairs + planarity"),
    (r"            st\.idx1\[q\] = i1;\n        \}\n    \}\n    __syncthreads\(\);", 23, "loss: consistency queries"),
    (r"for \(int q = tid; q < ncons; q \+= kPT\) \{ st\.idx2\[q\] = st\.idx1\[q\] \+ 1; st\.dist\[q\] = 0\.f; \}\n    \}\n    __syncthreads\(\);", 24, "loss: nearest pixel"),
    (r"    cs = block_sum\(cs, s_red\);", 25, "loss: consistency"),
]


def patch(dst):
    src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "indoor-nerf_amd", "csrc",
                       "priors_fused.hip")
    s = open(src).read()
    s = s.replace('#include "common.h"\n', '#include "common.h"\n#define PHASE(k) do { if (threadIdx.x == 0) '
                  'reinterpret_cast<uint64_t*>(a.members)[k] = wall_clock64(); } while (0)\n', 1)
    for rx, k, name in PHASES:
        m = list(re.finditer(rx, s))
        if len(m) != 1:   # an anchor of an older source
            print("skipped", name, len(m))
            continue
        stamp = f"PHASE({k});" if k not in (3, 40, 41) else ("PHASE(3 + it);" if k == 3 else f"PHASE({k} + 3 * it);")
        s = s[:m[0].end()] + "\n    " + stamp + s[m[0].end():]
    open(dst, "w").write(s)


def run(reps=20):
    import numpy as np
    import torch
    sys.path.insert(0, os.getcwd())
    from indoor_nerf_amd import _lib, priors  # noqa: F401
    dev = torch.device("cuda", 0)
    N = 4096
    g = torch.Generator().manual_seed(0)
    n = torch.randn(N, 3, generator=g)
    n[: N // 3] = torch.tensor([0.05, 0.02, 1.0]) + 0.1 * torch.randn(N // 3, 3, generator=g)
    n[N // 3: 2 * N // 3, 2] *= 0.1
    d = torch.rand(N, generator=g) * 3 + 0.5
    xy = torch.stack([torch.randint(0, 640, (N,), generator=g), torch.randint(0, 480, (N,), generator=g)], -1).float()
    d, n, xy = d.to(dev).requires_grad_(True), n.to(dev).requires_grad_(True), xy.to(dev)
    ws = torch.empty(int(_lib.load().nerf_priors_workspace_bytes(N)), dtype=torch.uint8, device=dev)
    off = ws.numel() - 3 * N * 4
    off -= off % 256
    rows = []
    for r in range(reps + 3):
        t, _ = priors.fused_structural_losses(d, n, xy, workspace=ws)
        torch.cuda.synchronize()
        st = ws[off:off + 80 * 8].view(torch.int64).cpu().numpy().astype(np.float64) / 100.0   # us
        if r >= 3:
            rows.append(st)
    st = np.mean(rows, 0)
    rnd = [(st[40 + 3 * it] - (st[2] if it == 0 else st[2 + it]), st[41 + 3 * it] - st[40 + 3 * it],
            st[3 + it] - st[41 + 3 * it]) for it in range(10)]
    print("k-means round split (points, 12 sums, centre update) us:", " ".join("%.2f/%.2f/%.2f" % r for r in rnd))
    prev = None
    for rx, k, name in PHASES:
        idx = list(range(3, 13)) if k == 3 else [k]
        for i in idx:
            if prev is not None and name != "prep: start" and name != "loss: start":
                print(f"{name if k != 3 else f'prep: k-means round {i - 3}':32s} {st[i] - st[prev]:7.2f} us")
            prev = i
    print(f"{'prep total':32s} {st[13] - st[0]:7.2f} us; loss total {st[25] - st[16]:7.2f} us")


if __name__ == "__main__":
    if sys.argv[1] == "--patch":
        patch(sys.argv[2])
    else:
        run()
