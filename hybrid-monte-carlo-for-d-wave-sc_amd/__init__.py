"""MI355X-native fermionic action/force path of DwaveHMC.jl.

Layout:
  csrc/      gfx950 HIP kernels + the C ABI (include/dwhmc.h) -> libdwhmc.so
  _lib.py    ctypes binding of the ABI
  context.py FermionContext: batched device handle
  hmc.py     the reference's hot-path API (ModelParameters ... hmc_sweep)
  simulation.py run_simulation (src/Simulation.jl): adaptive Nt, log, observables.csv
  replicas.py one-process-per-GPU replica driver (RCCL only gathers observables)

The directory name is not a Python identifier; import it through
`dwhmc_loader.load_package()` (repo root) or `importlib`.
"""
from .hmc import (ComputeCache, ModelParameters, ObservablesResult, SimulationState, calc_optimal_dt,
                  compute_forces, compute_total_energy, diagonalize_H_BdG, hmc_sweep, init_static_H,
                  initialize_cache, initialize_state, measure_observables, neighbour_tables,
                  refresh_momentum, standard_complex_normal, update_H_BdG, SpectrumResult,
                  measure_transport_and_spectra)
from .context import FermionContext, selftest_mfma, transport_grid
from .simulation import AdaptiveNt, SimulationResult, run_simulation, run_simulation_chains
from ._lib import DwhError, SpectrumGuardError, lib_path, load as load_library

__all__ = [
    "ComputeCache", "ModelParameters", "ObservablesResult", "SimulationState", "calc_optimal_dt",
    "compute_forces", "compute_total_energy", "diagonalize_H_BdG", "hmc_sweep", "init_static_H",
    "initialize_cache", "initialize_state", "measure_observables", "neighbour_tables",
    "refresh_momentum", "standard_complex_normal", "update_H_BdG", "FermionContext", "selftest_mfma",
    "DwhError", "SpectrumGuardError", "lib_path", "load_library", "AdaptiveNt", "SimulationResult",
    "run_simulation", "run_simulation_chains", "SpectrumResult", "measure_transport_and_spectra", "transport_grid",
]
