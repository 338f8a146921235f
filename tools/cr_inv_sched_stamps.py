#!/usr/bin/env python3
"""Phase stamps of the CR inversion launches in the library's own schedule
(VERDICT r04 next #2): a -DCR_STAMPS build of libdwhmc (build/stamps/,
hybrid-monte-carlo-for-d-wave-sc_amd/build.py --out ... -D CR_STAMPS) records
per-workgroup s_memtime phase stamps and s_memrealtime entry / exit times of
one inversion launch per factorisation (dwh_debug_cr_stamps), side-work and
guard workgroups included.  Prints, per inversion stage of the C3 plan: the
launch span (first entry to last exit, 100 MHz clock), when the inversion /
side / guard workgroups enter and leave, and the inversion workgroups' phase
split (wave 0's view, shader-clock ticks, median over workgroups).

Usage: python tools/cr_inv_sched_stamps.py [--L 32 --beta 16 --reps 5] [--json out.json]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

K_PHASES = {   # k_cr_inv_side<4> / k_cr_inv<4> (cr_inv_wg), stamp index -> phase ending there
    2: "load block (+ vmcnt)", 3: "pivot 0 inverse (wave 0)",
}
for kb in range(8):
    K_PHASES[4 + 3 * kb] = f"kb={kb}: barrier 1 (publish / wait)"
    K_PHASES[5 + 3 * kb] = f"kb={kb}: phase 1 (X = P^-1 A_kJ) + barrier 2"
    K_PHASES[6 + 3 * kb] = f"kb={kb}: phase 2, wave 0's part"
K_PHASES[28] = "store + ln|det| (+ vmcnt)"
INV0_PHASES = {2: "load A, B, R + barrier", 3: "Z = R B + barrier", 4: "S, S00^-1 (w0) + barrier",
               5: "P, Q; T, T^-1 (w3) + barrier", 6: "X01, X10, X00 + barrier", 7: "Y = Z conj X",
               28: "store + ln|det| (+ vmcnt)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=32)
    ap.add_argument("--beta", type=float, default=16.0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--lib", default=os.path.join(ROOT, "build", "stamps", "libdwhmc.so"))
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import dwhmc_loader
    m = dwhmc_loader.load_package()
    p = m.ModelParameters(a.L, a.L, 1.0, -0.35, -1.08, 1.0, 0.05, a.beta, 0.8, 1.0)
    st = m.initialize_state(p, np.random.default_rng(1000))
    ctx = m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table,
                           st.disorder_pot[None], lib_path=a.lib)
    ctx.set_pairing(st.Delta)
    for _ in range(3):
        ctx.factorize()
    ctx.synchronize()
    nwg = 2048
    out = np.zeros((nwg, 32), dtype=np.uint64)
    res = []
    stage = 0
    P = ctx.info["npoles"]
    print(f"L={a.L} beta={a.beta} poles={P} (stamp build: timings include the stamps' own cost)")
    while True:
        recs = []
        for _ in range(a.reps):
            out[:] = 0
            rc = ctx._lib.dwh_debug_cr_stamps(ctx._h, stage, out.ctypes.data_as(C.c_void_p), nwg)
            if rc != 0:
                break
            recs.append(out.copy())
        if not recs:
            break
        spans, kinds = [], {}
        phase = {}
        for o in recs:
            used = o[:, 31] > 0
            t0 = o[used, 0].astype(np.int64).min()
            t1 = o[used, 30].astype(np.int64).max()
            spans.append((t1 - t0) / 100.0)   # us (100 MHz)
            for kd, name in ((1, "inversion"), (2, "side"), (3, "guard")):
                sel = o[:, 31] == kd
                if sel.any():
                    ent = (o[sel, 0].astype(np.int64) - t0) / 100.0
                    ext = (o[sel, 30].astype(np.int64) - t0) / 100.0
                    k = kinds.setdefault(name, {"n": int(sel.sum()), "enter": [], "exit": [], "life": []})
                    k["enter"].append(np.median(ent))
                    k["exit"].append(np.median(ext))
                    k["life"].append(np.median(ext - ent))
                    k.setdefault("exit_max", []).append(ext.max())
            sel = o[:, 31] == 1
            st_ = o[sel].astype(np.int64)
            idx = [i for i in range(1, 30) if (st_[:, i] > 0).all()]
            for i0, i1 in zip(idx[:-1], idx[1:]):
                phase.setdefault(i1, []).append(float(np.median(st_[:, i1] - st_[:, i0])))
            phase.setdefault("total", []).append(float(np.median(st_[:, idx[-1]] - st_[:, idx[0]])))
        names = INV0_PHASES if stage == 0 and a.L == 32 else K_PHASES
        rec = {"stage": stage, "span_us": float(np.median(spans)),
               "groups": {k: {"n": v["n"], "enter_us": float(np.median(v["enter"])), "exit_us": float(np.median(v["exit"])),
                              "exit_max_us": float(np.median(v["exit_max"])), "life_us": float(np.median(v["life"]))}
                          for k, v in kinds.items()},
               "phases_ticks": {names.get(k, str(k)) if k != "total" else "total": float(np.median(v))
                                for k, v in phase.items()}}
        res.append(rec)
        print(f"\ninversion stage {stage}: launch span {rec['span_us']:.1f} us")
        for k, v in rec["groups"].items():
            print(f"  {k:9s} x{v['n']:4d}: enter {v['enter_us']:5.1f} us  exit {v['exit_us']:5.1f} (last {v['exit_max_us']:5.1f})"
                  f"  lifetime {v['life_us']:5.1f} us")
        for k, v in rec["phases_ticks"].items():
            print(f"  {k:44s} {v:8.0f}")
        stage += 1
    ctx.close()
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"L": a.L, "beta": a.beta, "poles": P, "clock": "phases: s_memtime ticks (shader clock); "
                       "enter/exit/span: s_memrealtime (100 MHz)", "stages": res}, f, indent=1)


if __name__ == "__main__":
    main()
