#!/usr/bin/env python3
"""Phase timeline of k_cr_gemm workgroups in one leapfrog-step factorisation
(diagnostic build with -DCR_GEMM_STAMPS: build/var/gstamps.so).

For every product stage of the L x L plan (read from DWHMC_CR_PLAN_DUMP), one
factorisation with that stage selected records per workgroup (wave 0):
realtime start/end (100 MHz) and shader-clock stamps at entry, descriptor
loaded, partials written to LDS (K loop + MFMA results), after the reduction
barrier, end (stores done).  Prints per stage: workgroups, launch span,
median workgroup lifetime and its split, and how many workgroups ran
concurrently on average.

Usage: python tools/gemm_stamps.py [--L 32] [--beta 16] [--lib build/var/gstamps.so]
"""
import argparse
import ctypes as C
import os
import re
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=32)
    ap.add_argument("--beta", type=float, default=16.0)
    ap.add_argument("--lib", default=os.path.join(ROOT, "build", "var", "gstamps.so"))
    a = ap.parse_args()
    import dwhmc_loader
    m = dwhmc_loader.load_package()
    p = m.ModelParameters(a.L, a.L, 1.0, -0.35, -1.08, 1.0, 0.05, a.beta, 0.8, 1.0)
    st = m.initialize_state(p, np.random.default_rng(1000))
    os.environ["DWHMC_CR_PLAN_DUMP"] = "1"
    tmp = tempfile.TemporaryFile(mode="w+")
    saved = os.dup(2)
    os.dup2(tmp.fileno(), 2)
    try:
        ctx = m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table,
                               st.disorder_pot, lib_path=a.lib)
    finally:
        os.dup2(saved, 2)
        os.environ.pop("DWHMC_CR_PLAN_DUMP")
    tmp.seek(0)
    plan = tmp.read()
    lib = C.CDLL(os.path.abspath(a.lib))
    nbatch = ctx.info["nchains"] * ctx.info["npoles"]
    stages = []
    for line in plan.splitlines():
        mm = re.match(r"cr stage\s+(\d+): gemm .*ntmax=(\d+).*ntiles=(\d+)", line)
        if mm:
            stages.append((int(mm.group(1)), int(mm.group(2)), int(mm.group(3)) * nbatch))
        elif re.match(r"cr stage\s+(\d+): inv", line):
            stages.append((int(line.split()[2].rstrip(":")), -1, 0))
    ctx.set_pairing(st.Delta)
    ctx.factorize()
    print(f"L={a.L} beta={a.beta:g} poles={ctx.info['npoles']}  (clock = shader clock cycles; span in us)")
    print("stage nt    tiles   WGs  span_us  life_cyc  desc  kloop  barrier  store   conc")
    for idx, nt, total in stages:
        if nt < 0:
            print(f"{idx:5d} inversion")
            continue
        nwg = total   # KSPLIT 4: one 16x16 tile per workgroup
        lib.dwh_debug_gemm_stamps_select(C.c_int(total))
        ctx.set_pairing(st.Delta)
        ctx.factorize()
        buf = np.zeros((min(nwg, 65536), 8), dtype=np.uint64)
        lib.dwh_debug_gemm_stamps_read(buf.ctypes.data_as(C.c_void_p), C.c_int(buf.shape[0]))
        lib.dwh_debug_gemm_stamps_select(C.c_int(-1))
        b = buf.astype(np.float64)
        rt0, rt1 = b[:, 0], b[:, 6]
        span = (rt1.max() - rt0.min()) / 100.0      # 100 MHz -> us
        life = b[:, 5] - b[:, 1]
        desc = b[:, 2] - b[:, 1]
        kl = b[:, 3] - b[:, 2]
        bar = b[:, 4] - b[:, 3]
        sto = b[:, 5] - b[:, 4]
        conc = ((rt1 - rt0).sum() / 100.0) / span if span > 0 else float("nan")
        print(f"{idx:5d} {nt:2d} {total:8d} {nwg:5d} {span:8.1f} {np.median(life):9.0f} {np.median(desc):5.0f} "
              f"{np.median(kl):6.0f} {np.median(bar):8.0f} {np.median(sto):6.0f} {conc:6.0f}")
    ctx.close()


if __name__ == "__main__":
    main()
