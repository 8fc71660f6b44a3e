"""Build libpdvc_hip.so (all HIP kernels + the C ABI) for gfx950 with hipcc, in-tree.

    python dense-video-captioning_amd/build_native.py [--force]

The library lands in dense-video-captioning_amd/lib/ (git-ignored, travels with the tree to the GPU box).
"""
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(HERE, "lib", "libpdvc_hip.so")
ARCH = os.environ.get("PDVC_OFFLOAD_ARCH", "gfx950")


def sources():
    return sorted(glob.glob(os.path.join(HERE, "csrc", "*.hip")) + glob.glob(os.path.join(HERE, "csrc", "*.cpp")))


def headers():
    return sorted(glob.glob(os.path.join(HERE, "csrc", "*.h")) + glob.glob(os.path.join(ROOT, "include", "*.h")))


def build(force=False, verbose=True):
    srcs = sources()
    deps = srcs + headers() + [os.path.abspath(__file__)]
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= max(os.path.getmtime(p) for p in deps):
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objs = []
    objdir = os.path.join(HERE, "build", ARCH)
    os.makedirs(objdir, exist_ok=True)
    procs = []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        if not force and os.path.exists(o) and os.path.getmtime(o) >= max(os.path.getmtime(p) for p in [s] + headers()):
            continue
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function",
               "-I", os.path.join(ROOT, "include"), "-I", os.path.join(HERE, "csrc"), "-c", s, "-o", o]
        if s.endswith(".cpp"):  # host-only C++ (status plumbing)
            cmd[1:1] = ["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    failed = False
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed = True
            sys.stderr.write(out.decode(errors="replace"))
        elif verbose and out:
            sys.stderr.write(out.decode(errors="replace"))
    if failed:
        raise RuntimeError("hipcc failed")
    subprocess.check_call([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT] + objs)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
