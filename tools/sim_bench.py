"""Reference-style run on the device: run_simulation (src/Simulation.jl:34-236)
at L x L with transport every measurement sweep (measure_transport_freq = 1),
timing the measurement phase per sweep for transport_batch = 1 and 16.
python tools/sim_bench.py [L] [n_measure]"""
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    nm = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    import dwhmc_loader
    m = dwhmc_loader.load_package()
    sim = m.simulation
    p = m.ModelParameters(L, L, 1.0, -0.35, -1.08, 1.0, 0.1, 16.0, 0.8, 1.0)
    def run(n, batch):
        with tempfile.TemporaryDirectory() as d:
            t0 = time.perf_counter()
            sim.run_simulation(p, d, n_therm=4, n_measure=n, measure_transport_freq=1, bin_size=4, verbose=False,
                               rng=np.random.default_rng(1), transport_batch=batch)
            return time.perf_counter() - t0

    run(16, 16)   # warm-up: library load, context creation, kernels' first launches
    for batch in (1, 16):
        t_th = run(0, batch)
        el = run(nm, batch) - t_th
        print(f"L={L} transport every sweep, transport_batch={batch}: {1e3 * el / nm:.2f} ms per measurement sweep "
              f"({nm} sweeps, HMC + transport + files; thermalisation subtracted)", flush=True)


if __name__ == "__main__":
    main()
