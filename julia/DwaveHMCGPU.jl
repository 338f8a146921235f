# DwaveHMCGPU.jl — Julia `ccall` binding of libdwhmc.so (include/dwhmc.h).
#
# Drop-in for the hot path of DwaveHMC.jl: `GPUCache` replaces `ComputeCache`
# and the methods below shadow init_static_H!/update_H_BdG!/diagonalize_H_BdG!/
# compute_forces!/compute_total_energy/hmc_sweep! for it, with the reference's
# argument order and mutation semantics (src/Hamiltonian.jl, src/Observables.jl,
# src/HMC.jl).  Not executable in this image (no Julia, SURVEY.md F4); the
# ABI it binds is exercised through ctypes by tests/test_gpu_parity.py.
module DwaveHMCGPU

using DwaveHMC
using Random
import DwaveHMC: init_static_H!, update_H_BdG!, diagonalize_H_BdG!, compute_forces!,
                 compute_total_energy, hmc_sweep!, measure_transport_and_spectra

const libdwhmc = get(ENV, "DWHMC_LIB", joinpath(@__DIR__, "..", "hybrid-monte-carlo-for-d-wave-sc_amd", "libdwhmc.so"))

struct DwhError <: Exception
    code::Cint
    msg::String
end

function check(ctx::Ptr{Cvoid}, rc::Cint)
    rc == 0 && return nothing
    msg = unsafe_string(ccall((:dwh_last_error, libdwhmc), Cstring, (Ptr{Cvoid},), ctx))
    rc == -1 && throw(ArgumentError(msg))
    throw(DwhError(rc, msg))
end

"""GPU-resident replacement of ComputeCache (src/Types.jl:145-212)."""
mutable struct GPUCache
    ctx::Ptr{Cvoid}
    forces::Matrix{ComplexF64}
    E_fermion::Float64
    device::Int32
    delta_cap::Float64
end

function GPUCache(p::ModelParameters; device::Integer=0, delta_cap::Real=2.0)
    c = GPUCache(C_NULL, zeros(ComplexF64, p.N, 2), 0.0, Int32(device), Float64(delta_cap))
    finalizer(c) do c
        c.ctx == C_NULL || ccall((:dwh_destroy, libdwhmc), Cvoid, (Ptr{Cvoid},), c.ctx)
        c.ctx = C_NULL
    end
    return c
end

# src/Hamiltonian.jl:10-47 — the disorder is consumed here, as in the reference
function init_static_H!(cache::GPUCache, p::ModelParameters, state::SimulationState)
    cache.ctx == C_NULL || ccall((:dwh_destroy, libdwhmc), Cvoid, (Ptr{Cvoid},), cache.ctx)
    ref = Ref{Ptr{Cvoid}}(C_NULL)
    GC.@preserve p state begin
        rc = ccall((:dwh_create_batched, libdwhmc), Cint,
                   (Ref{Ptr{Cvoid}}, Int64, Int64, Float64, Float64, Float64, Float64, Float64,
                    Ptr{Int64}, Ptr{Int64}, Int64, Ptr{Float64}, Float64, Int32),
                   ref, p.Lx, p.Ly, p.t, p.tp, p.μ, p.β, p.J, p.nn_table, p.nnn_table,
                   1, state.disorder_pot, cache.delta_cap, cache.device)
    end
    check(C_NULL, rc)
    cache.ctx = ref[]
    return nothing
end

# src/Hamiltonian.jl:55-86 — Δ is Julia's column-major N×2 ComplexF64 = the ABI layout
function update_H_BdG!(cache::GPUCache, p::ModelParameters, state::SimulationState)
    GC.@preserve state check(cache.ctx, ccall((:dwh_update_pairing, libdwhmc), Cint,
                                              (Ptr{Cvoid}, Ptr{ComplexF64}), cache.ctx, state.Δ))
end

# src/Hamiltonian.jl:96-114 replacement (pole-expanded no-pivot LU, no eigenpairs)
function diagonalize_H_BdG!(cache::GPUCache, p::ModelParameters)
    check(cache.ctx, ccall((:dwh_factorize, libdwhmc), Cint, (Ptr{Cvoid},), cache.ctx))
    ef = Ref{Float64}(0.0)
    check(cache.ctx, ccall((:dwh_fermion_energy, libdwhmc), Cint, (Ptr{Cvoid}, Ref{Float64}), cache.ctx, ef))
    cache.E_fermion = ef[]
    return nothing
end

# src/Observables.jl:14-62
function compute_forces!(cache::GPUCache, p::ModelParameters, state::SimulationState)
    GC.@preserve state cache check(cache.ctx, ccall((:dwh_forces, libdwhmc), Cint,
                                                    (Ptr{Cvoid}, Ptr{ComplexF64}, Ptr{ComplexF64}),
                                                    cache.ctx, state.Δ, cache.forces))
end

# src/HMC.jl:12-41
function compute_total_energy(cache::GPUCache, p::ModelParameters, state::SimulationState)
    GC.@preserve state check(cache.ctx, ccall((:dwh_set_state, libdwhmc), Cint,
                                              (Ptr{Cvoid}, Ptr{ComplexF64}, Ptr{ComplexF64}),
                                              cache.ctx, state.Δ, state.π))
    h = Ref{Float64}(0.0)
    check(cache.ctx, ccall((:dwh_total_energy, libdwhmc), Cint, (Ptr{Cvoid}, Float64, Ref{Float64}),
                           cache.ctx, p.mass, h))
    return h[]
end

# src/HMC.jl:71-144: the reference's own RNG draws (randn!, rand) are taken
# here and handed to the device, so a seeded Julia RNG reproduces a run.
function hmc_sweep!(cache::GPUCache, p::ModelParameters, state::SimulationState; Nt::Int, dt::Float64)
    noise = randn(ComplexF64, p.N, 2)
    u = Ref(rand())
    acc = Ref{UInt8}(0)
    dH = Ref{Float64}(0.0)
    GC.@preserve state noise begin
        check(cache.ctx, ccall((:dwh_set_state, libdwhmc), Cint,
                               (Ptr{Cvoid}, Ptr{ComplexF64}, Ptr{ComplexF64}), cache.ctx, state.Δ, C_NULL))
        check(cache.ctx, ccall((:dwh_hmc_sweep, libdwhmc), Cint,
                               (Ptr{Cvoid}, Ptr{ComplexF64}, Ref{Float64}, Int64, Float64, Float64,
                                Ref{UInt8}, Ref{Float64}),
                               cache.ctx, noise, u, Nt, dt, p.mass, acc, dH))
        check(cache.ctx, ccall((:dwh_get_state, libdwhmc), Cint,
                               (Ptr{Cvoid}, Ptr{ComplexF64}, Ptr{ComplexF64}), cache.ctx, state.Δ, state.π))
    end
    return acc[] != 0, dH[]
end

# src/Observables.jl:314-526 on the device (eigenpairs by rocSOLVER, sums in HIP
# kernels) for the Δ the context holds; same SpectrumResult.
function measure_transport_and_spectra(cache::GPUCache, p::ModelParameters)
    nw, nd = Ref{Int64}(0), Ref{Int64}(0)
    check(C_NULL, ccall((:dwh_transport_grid, libdwhmc), Cint,
                        (Float64, Float64, Float64, Ref{Int64}, Ref{Int64}), p.η, p.Δω, p.ω_max, nw, nd))
    st, dc = Ref{Float64}(0.0), Ref{Float64}(0.0)
    σ, dos, dos_AN = zeros(nw[]), zeros(nd[]), zeros(nd[])
    ak = zeros(p.Lx, p.Ly)
    check(cache.ctx, ccall((:dwh_measure_transport, libdwhmc), Cint,
                           (Ptr{Cvoid}, Int64, Float64, Float64, Float64, Ref{Float64}, Ref{Float64},
                            Ptr{Float64}, Int64, Ptr{Float64}, Ptr{Float64}, Int64, Ptr{Float64}),
                           cache.ctx, 0, p.η, p.Δω, p.ω_max, st, dc, σ, nw[], dos, dos_AN, nd[], ak))
    return DwaveHMC.SpectrumResult(st[], dc[], collect(p.ω_min:p.Δω:p.ω_max), σ,
                                   collect(-p.ω_max:p.Δω:p.ω_max), dos, dos_AN, ak)
end

end # module
