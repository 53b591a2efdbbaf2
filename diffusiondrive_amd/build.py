"""Build ``libddmi.so`` (HIP kernels + C-ABI runtime) in-tree for gfx950 with hipcc.

Usage: ``python -m diffusiondrive_amd.build`` (or ``__graft_entry__.build()``). Objects are
cached under ``diffusiondrive_amd/_build`` and rebuilt when a source or header changes. The
shared library lands next to this file so it travels to the GPU box with the repo snapshot.
"""
import hashlib
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
BUILD = os.path.join(HERE, "_build")
ARCH = os.environ.get("DDMI_ARCH", "gfx950")
# DDMI_BUILD_VARIANT=stamps: a diagnostic library (libddmi_stamps.so, load it with DDMI_LIB) whose decoder
# megakernel records per-phase clock stamps (tools/debug/mk_stamps.py); the product library has none.
# DDMI_BUILD_VARIANT=x5st / x6st: conv_x5 / conv_x6 per-workgroup phase stamps (tools/micro/build_conv_bench.sh)
VARIANT = os.environ.get("DDMI_BUILD_VARIANT", "")
LIB = os.path.join(HERE, "libddmi.so") if not VARIANT else os.path.join(HERE, "_variants", f"libddmi_{VARIANT}.so")
VARIANT_FLAGS = {"": [], "stamps": ["-DDDMI_MK_STAMPS"], "nopv": ["-DDDMI_MK_STAMPS", "-DDDMI_MK_NOPV"], "x5st": ["-DDDMI_X5_STAMPS"], "x6st": ["-DDDMI_X6_STAMPS"], "nobar": ["-DDDMI_X5_NOBAR", "-DDDMI_X5_STAMPS"], "x6nb": ["-DDDMI_X6_NOBAR"], "vust": ["-DDDMI_VU_STAMPS"], "dbg": ["-g", "-DDDMI_SEGV_TRACE"]}[VARIANT]
SOURCES = ["conv_gemm.hip", "conv_x3.hip", "conv_x5.hip", "conv_x6.hip", "elementwise.hip", "decoder.hip", "decoder_mk.hip", "tfdec_mk.hip", "bevproj.hip", "value_proj.hip", "attention.hip", "gpt_tail.hip", "stem_pool.hip", "features.hip", "train_loss.hip", "weights.cpp", "runtime.cpp", "ops_abi.cpp"]
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-I", CSRC, "-I", INCLUDE] + VARIANT_FLAGS
# Elementwise / decoder arithmetic must round like PyTorch-CPU's separate mul and add kernels
# (no a*b+c -> fma contraction): the DDIM / norm_odo / bilinear-weight chains feed the BEV
# sampling positions, which are sensitive at the 1e-5 m level.
PER_SOURCE_FLAGS = {"decoder.hip": ["-ffp-contract=off"], "train_loss.hip": ["-ffp-contract=off"], "decoder_mk.hip": ["-ffp-contract=off"], "bevproj.hip": ["-ffp-contract=off"], "tfdec_mk.hip": ["-ffp-contract=off"], "elementwise.hip": ["-ffp-contract=off"],
                    "runtime.cpp": ["-ffp-contract=off"]}


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the ddmi HIP library cannot be built")


def _headers_digest():
    h = hashlib.sha256()
    for d in (CSRC, INCLUDE):
        for f in sorted(os.listdir(d)):
            if f.endswith(".h"):
                with open(os.path.join(d, f), "rb") as fh:
                    h.update(fh.read())
    return h.hexdigest()[:16]


def _compile(hipcc, src, hdr):
    path = os.path.join(CSRC, src)
    with open(path, "rb") as fh:
        flags = FLAGS + PER_SOURCE_FLAGS.get(src, [])
        digest = hashlib.sha256(fh.read() + hdr.encode() + " ".join(flags).encode()).hexdigest()[:16]
    obj = os.path.join(BUILD, f"{src}.{digest}.o")
    if not os.path.exists(obj):
        cmd = [hipcc, *flags, "-c", path, "-o", obj + ".tmp"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
        os.replace(obj + ".tmp", obj)
    return obj


def build(verbose: bool = True) -> str:
    hipcc = _hipcc()
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    hdr = _headers_digest()
    with ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(lambda s: _compile(hipcc, s, hdr), SOURCES))
    key = hashlib.sha256("".join(objs).encode()).hexdigest()[:16]
    stamp = os.path.join(BUILD, f"lib{VARIANT}.stamp")
    if os.path.exists(LIB) and os.path.exists(stamp) and open(stamp).read() == key:
        return LIB
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB + ".tmp", *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(LIB + ".tmp", LIB)
    with open(stamp, "w") as fh:
        fh.write(key)
    if verbose:
        print(f"[ddmi] built {LIB}", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    build()
