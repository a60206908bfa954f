"""Build libmk.so (gfx950) in-tree with hipcc.  Used by __graft_entry__.build()."""
import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_PATH = os.path.join(PKG_DIR, "libmk.so")
SOURCES = ["mk_linalg.hip", "mk_mcmc.hip", "mk_init.hip", "mk_post.hip", "mk_api.hip", "mk_multi.hip", "mk_watch.hip", "mk_rsample.cpp"]
HEADERS = ["mk_common.hpp", "mk_types.hpp", "mk_gemm.hpp", "mk_corr.hpp", "mk_kernels.hpp", "mk_internal.hpp"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wno-unused-value",
         "-Wno-unused-result"]


def _stale():
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(PKG_DIR, "..", "include", "mk.h"))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False, out=None, defines=()):
    """libmk.so in-tree; out / defines (e.g. ["MK_TRI_SKIP=0"]): an A/B variant elsewhere, loaded
    through MK_LIB (tools only -- the package always loads the in-tree library by default)."""
    lib_path = out or LIB_PATH
    if out is None and not force and not _stale():
        return LIB_PATH
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objs = []
    procs = []
    tag = "" if out is None else ".variant"
    for src in SOURCES:
        obj = os.path.join(CSRC, os.path.splitext(src)[0] + tag + ".o")
        cmd = [hipcc] + FLAGS + ["-D" + d for d in defines] + ["-c", os.path.join(CSRC, src), "-o", obj]
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        objs.append(obj)
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            sys.stderr.write(out.decode(errors="replace"))
            raise RuntimeError("hipcc failed: " + " ".join(cmd))
        if verbose and out:
            sys.stderr.write(out.decode(errors="replace"))
    tmp = lib_path + ".tmp"
    cmd = [hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp] + objs + ["-ldl"]
    subprocess.check_call(cmd)
    os.replace(tmp, lib_path)
    for o in objs:
        os.remove(o)
    return lib_path


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
