import ctypes as C, os, sys, numpy as np
sys.path.insert(0, os.getcwd())
import dwhmc_loader
m = dwhmc_loader.load_package()
p = m.ModelParameters(32, 32, 1.0, -0.35, -1.08, 1.0, 0.05, 16.0, 0.8, 1.0)
st = m.initialize_state(p, np.random.default_rng(1000))
ctx = m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table, st.disorder_pot[None], lib_path="build/stamps/libdwhmc.so")
ctx.set_pairing(st.Delta); ctx.factorize(); ctx.synchronize()
out = np.zeros((2048, 32), dtype=np.uint64)
for s in range(3):
    out[:] = 0
    rc = ctx._lib.dwh_debug_cr_stamps(ctx._h, s, out.ctypes.data_as(C.c_void_p), 2048)
    print("stage", s, "rc", rc, "nonzero rows", int((out != 0).any(1).sum()), "kinds", np.unique(out[:, 31]), flush=True)
    if rc: print(ctx._lib.dwh_last_error(ctx._h))
