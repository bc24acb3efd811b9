#!/usr/bin/env python3
"""Build the native gfx950 kernel library and the C++ runtime helpers, in-tree.

    python build_native.py [--jobs N] [--arch gfx950] [--debug]

Outputs (git-ignored, but shipped to the GPU box with the tree):
    trustworthy_dl/_native/libtdl_kernels.so   HIP kernels (csrc/*.hip), C ABI, loaded by ops/_lib.py
    trustworthy_dl/_native/libtdl_runtime.so   host C++ runtime (csrc/runtime/*.cpp), loaded by runtime/native.py
Incremental: a translation unit is rebuilt only when it or a header is newer than its object.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(ROOT, "csrc")
OUT_DIR = os.path.join(ROOT, "trustworthy_dl", "_native")
BUILD_DIR = os.path.join(ROOT, "build", "native")
NO_NAN_FLAGS = {"attention.hip": ["-fno-honor-nans"]}
AGPR_FORM = {"gemm.hip"}


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm required)")


def _newer(src: str, obj: str, deps) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return os.path.getmtime(src) > t or any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    return p.returncode, " ".join(cmd), p.stdout


def build(arch: str = "gfx950", jobs: int = 8, debug: bool = False, verbose: bool = False) -> dict:
    os.makedirs(OUT_DIR, exist_ok=True)
    os.makedirs(BUILD_DIR, exist_ok=True)
    cc = hipcc()
    opt = ["-O1", "-g"] if debug else ["-O3"]
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    kernel_srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    rt_srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    rt_headers = glob.glob(os.path.join(CSRC, "runtime", "*.h"))

    jobs_list = []
    kobjs, robjs = [], []
    for src in kernel_srcs:
        obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
        kobjs.append(obj)
        if _newer(src, obj, headers):
            # MFMA accumulators in ArchVGPRs: the default AGPR form shuttles every softmax / epilogue
            # read through v_accvgpr_read/write and pushed the attention forward past 256 registers
            # (one wave per SIMD); the VGPR form holds it at 140 (three waves per SIMD)
            # the persistent GEMM keeps its 256 accumulators per lane in AGPRs (one wave per SIMD,
            # 512 registers): it is built in the default AGPR form
            form = [] if os.path.basename(src) in AGPR_FORM else ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]
            # attention softmax: scores are finite or -inf, never NaN; without NaN semantics fmax
            # of an MFMA result needs no canonicalising v_max in front of it (csrc/attention.hip)
            form += NO_NAN_FLAGS.get(os.path.basename(src), [])
            jobs_list.append([cc, f"--offload-arch={arch}", "-std=c++17", "-fPIC", *opt, "-munsafe-fp-atomics",
                              *form, "-I", CSRC, "-c", src, "-o", obj])
    for src in rt_srcs:
        obj = os.path.join(BUILD_DIR, "rt_" + os.path.basename(src) + ".o")
        robjs.append(obj)
        if _newer(src, obj, rt_headers):
            jobs_list.append(["g++", "-std=c++17", "-fPIC", "-O2", "-Wall", "-pthread",
                              "-I", os.path.join(CSRC, "runtime"), "-c", src, "-o", obj])

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for rc, cmd, out in ex.map(_run, jobs_list):
            if verbose or rc != 0:
                print(cmd)
                print(out)
            if rc != 0:
                raise RuntimeError(f"compile failed: {cmd}")

    outputs = {}
    if kobjs:
        lib = os.path.join(OUT_DIR, "libtdl_kernels.so")
        if not os.path.exists(lib) or any(os.path.getmtime(o) > os.path.getmtime(lib) for o in kobjs):
            rc, cmd, out = _run([cc, f"--offload-arch={arch}", "-shared", "-fPIC", *kobjs, "-o", lib + ".tmp"])
            if rc != 0:
                print(cmd)
                print(out)
                raise RuntimeError("link failed (kernels)")
            os.replace(lib + ".tmp", lib)
        outputs["kernels"] = lib
    if robjs:
        lib = os.path.join(OUT_DIR, "libtdl_runtime.so")
        if not os.path.exists(lib) or any(os.path.getmtime(o) > os.path.getmtime(lib) for o in robjs):
            rc, cmd, out = _run(["g++", "-shared", "-fPIC", "-pthread", *robjs, "-o", lib + ".tmp"])
            if rc != 0:
                print(cmd)
                print(out)
                raise RuntimeError("link failed (runtime)")
            os.replace(lib + ".tmp", lib)
        outputs["runtime"] = lib
    return outputs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default=os.environ.get("PYTORCH_ROCM_ARCH", "gfx950"))
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    outs = build(a.arch, a.jobs, a.debug, a.verbose)
    for k, v in outs.items():
        print(f"{k}: {v}")


if __name__ == "__main__":
    sys.exit(main())
