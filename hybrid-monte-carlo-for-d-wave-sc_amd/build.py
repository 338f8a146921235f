"""Build libdwhmc.so (gfx950) in-tree with hipcc.

The shared library is the drop-in boundary (include/dwhmc.h); it links only the
HIP runtime, no torch.  Called by __graft_entry__.build() and lazily by the
ctypes binding when the .so is missing or older than its sources.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libdwhmc.so")
SOURCES = [os.path.join(CSRC, "dwhmc_kernels.hip"), os.path.join(CSRC, "dwhmc_cr.hip"), os.path.join(CSRC, "dwhmc_cr_sparse.hip"),
           os.path.join(CSRC, "dwhmc_eig.hip"), os.path.join(CSRC, "dwhmc_gemm.hip"),
           os.path.join(CSRC, "dwhmc_transport.hip"), os.path.join(CSRC, "dwhmc_qeig.hip"),
           os.path.join(CSRC, "dwhmc_api.cpp")]
# rocSOLVER (zheevd for an order above kEigMaxN, zheev as the re-solve of a
# non-finite result) is the
# only vendor library the measurement path can call; every product runs on the
# library's own MFMA kernel (dwhmc_gemm.hip).  rocBLAS is linked for the
# rocsolver handle only.
LIBS = ["-L/opt/rocm/lib", "-lrocsolver", "-lrocblas", "-Wl,-rpath,/opt/rocm/lib"]
DEPS = SOURCES + [os.path.join(CSRC, "dwhmc_internal.h"), os.path.join(CSRC, "dwhmc_device.h"),
                  os.path.join(CSRC, "pole_table.inc"), os.path.join(CSRC, "pole_table_eps5e-12.inc"),
                  os.path.join(ROOT, "include", "dwhmc.h")]
# gfx950 only: several kernels use more than the 64 KiB of LDS per workgroup
# earlier CDNA parts allow (k_gemm<complex> 66.5 KiB, k_cr_inv0_96 ~119 KiB),
# and the tiling is sized for CDNA4's 160 KiB per CU
ARCH = "gfx950"
if os.environ.get("DWHMC_OFFLOAD_ARCH", ARCH) != ARCH:
    raise SystemExit(f"libdwhmc targets gfx950 (MI355X) only; DWHMC_OFFLOAD_ARCH="
                     f"{os.environ['DWHMC_OFFLOAD_ARCH']} is not supported")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    return "hipcc"


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in DEPS if os.path.exists(p))


def build(force: bool = False, verbose: bool = False, out: str = LIB, defines=()) -> str:
    """defines: extra -D flags for A/B builds of kernel variants (tools/ab_bench.py
    loads such a build through DWHMC_LIB); the default build uses none."""
    if not force and out == LIB and not needs_build():
        return LIB
    tmp = out + ".tmp"
    # kernel arguments preloaded into SGPRs (gfx950): a launch's first loads no
    # longer wait for the kernarg s_load (C3 -1.8 %, C2 -4.1 % per leapfrog step,
    # profiles/r03_exp_kernarg_preload.txt); MFMA accumulators in VGPRs instead
    # of AGPRs: the register inversions mix MFMA tiles and VALU pivot steps, and
    # drop ~90 % of their accvgpr copies (C3 -2.0 %,
    # profiles/r03_exp_mfma_vgpr_form.txt)
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-mllvm", "-amdgpu-kernarg-preload-count=16", "-mllvm", "-amdgpu-mfma-vgpr-form",
           "-Wall", "-Wno-unused-result", f"-I{os.path.join(ROOT, 'include')}",
           *[f"-D{d}" for d in defines], *SOURCES, *LIBS, "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--out", default=LIB)
    ap.add_argument("-D", dest="defines", action="append", default=[])
    a = ap.parse_args()
    print(build(force=a.force or a.out != LIB, verbose=True, out=a.out, defines=a.defines))
