#!/usr/bin/env python3
"""Build a variant of libnerfhip.so with extra -D flags into build/variants/<name>/libnerfhip.so, for
A/B timing on the GPU (NERF_HIP_LIB=<path>). Usage:
  build_variant.py NAME [--rev GITREV] [--patch FILE.diff] [-Dflags...]
--rev: build the sources of that revision, checked out into a temporary worktree; --patch: apply a
unified diff (paths relative to the repo root, tools/variants/*.diff) to a temporary copy of
indoor-nerf_amd/csrc first — diagnostic and A/B variants live there, not in the shipped kernels."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402


def main():
    name, defs = sys.argv[1], sys.argv[2:]
    out = os.path.join(ROOT, "build", "variants", name)
    os.makedirs(out, exist_ok=True)
    srcs = g._sources()
    patch = None
    if "--patch" in defs:
        k = defs.index("--patch")
        patch = os.path.abspath(defs[k + 1])
        defs = defs[:k] + defs[k + 2:]
    if defs[:1] == ["--rev"]:
        rev, defs = defs[1], defs[2:]
        wt = os.path.join("/tmp", "nerf_variant_" + name)
        subprocess.run(["git", "-C", ROOT, "worktree", "remove", "--force", wt], capture_output=True)
        subprocess.run(["git", "-C", ROOT, "worktree", "add", "--detach", wt, rev], check=True, capture_output=True)
        csrc = os.path.join(wt, "indoor-nerf_amd", "csrc")
        srcs = sorted(os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith((".hip", ".cpp")))
    if patch is not None:
        import shutil
        tmp = os.path.join("/tmp", "nerf_variant_patch_" + name)
        shutil.rmtree(tmp, ignore_errors=True)
        csrc0 = os.path.dirname(srcs[0])
        shutil.copytree(csrc0, os.path.join(tmp, "indoor-nerf_amd", "csrc"))
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))   # csrc includes ../../include
        subprocess.run(["patch", "-p1", "-d", tmp, "-i", patch], check=True)
        csrc = os.path.join(tmp, "indoor-nerf_amd", "csrc")
        srcs = [os.path.join(csrc, os.path.basename(f)) for f in srcs]
    cmds, objs = [], []
    for src in srcs:
        obj = os.path.join(out, os.path.basename(src) + ".o")
        objs.append(obj)
        cmds.append([g.HIPCC] + g.HIP_FLAGS + g.EXTRA_FLAGS.get(os.path.basename(src), []) + defs + ["-c", src, "-o", obj])
    with ThreadPoolExecutor(max_workers=8) as ex:
        list(ex.map(g._run, cmds))
    lib = os.path.join(out, "libnerfhip.so")
    subprocess.run([g.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib] + objs, check=True)
    print(lib)


if __name__ == "__main__":
    main()
