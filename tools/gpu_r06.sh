#!/bin/bash
# Round-6 GPU passes: bash tools/gpu_r06.sh TAG step [step ...]
#   suite   full `pytest -m gpu`
#   driver  the driver's bench command only
#   bench   the driver's command + C3 x200 + C2 + C5
#   sq3     instruction-class / issue counters of the C3 bench (tools/pmc_sq3.sh)
#   sq      SQ / MFMA-busy counters (tools/pmc_sq.sh) + the f64 MFMA peak micro
#   prof    rocprofv3 kernel stats + PMC traffic passes (tools/profile_round.sh) + step trace
#   profc2  rocprofv3 kernel stats of the C2 bench (PROF_CFG / PROF_STEPS: another config)
#   ab      tools/ab_bench.py in-process A/B (AB_VARIANTS, AB_ARGS, AB_TAG)
#   parity  a GPU parity subset (PARITY_K)
#   trans   transport timing (single measurement + snapshot batches)
# Every GPU step runs under its own timeout; the first failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
summ() {
  python - "$@" <<'PY'
import json, sys, os
for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(os.path.basename(f), round(d["value"], 1), "steps/s", "poles", d["config"]["poles"],
              "frac", round((d.get("roofline") or {}).get("frac") or 0, 3), "alg_frac", d.get("alg_frac_of_peak"),
              "asm_us", (d.get("assembly") or {}).get("avg_launch_us"))
    except Exception as e:
        print(f, e)
PY
}
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    suite)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 450 --timeout-method thread \
        > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
      tail -3 "$O/tests.log" ;;
    driver)
      timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.json" 2> "$O/bench_driver.err" \
        || { tail -20 "$O/bench_driver.err"; exit 1; }
      summ "$O/bench_driver.json" ;;
    bench)
      timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.json" 2> "$O/bench_driver.err" \
        || { tail -20 "$O/bench_driver.err"; exit 1; }
      timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-c1 \
        > "$O/bench_C3_200.json" 2> "$O/bench_C3_200.err" || exit 1
      timeout -k 10 300 python -u bench.py --config C2 --steps 200 --warmup 20 --no-cpu-baseline --no-c1 \
        > "$O/bench_C2.json" 2> "$O/bench_C2.err" || exit 1
      timeout -k 10 300 python -u bench.py --config C5 --steps 40 --warmup 8 --no-cpu-baseline --no-c1 \
        > "$O/bench_C5.json" 2> "$O/bench_C5.err" || exit 1
      summ "$O"/bench_*.json ;;
    sq3)
      bash tools/pmc_sq3.sh "$TAG" || exit 1 ;;
    sq)
      bash tools/pmc_sq.sh "$TAG" || exit 1
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_f64_peak.hip -o "$O/mfma_f64_peak" || exit 1
      timeout -k 10 60 "$O/mfma_f64_peak" > "$O/mfma_f64_peak.txt" 2>&1 || exit 1
      cat "$O/mfma_f64_peak.txt"
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
        SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/peak_pmc" -o run -- "$O/mfma_f64_peak" \
        > "$O/peak_pmc.log" 2>&1) || exit 1
      rm -f "$O/mfma_f64_peak" ;;
    prof)
      bash tools/profile_round.sh "$TAG" r06 || exit 1
      python3 tools/trace_step.py "$R/gpurun_out/prof_$TAG/stats/run_kernel_trace.csv" > "$O/step.txt" || exit 1
      rm -f "$R/gpurun_out/prof_$TAG/stats/run_kernel_trace.csv" ;;
    profc2)
      (export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/profc2" -o run -- \
        python3 bench.py --config ${PROF_CFG:-C2} --steps ${PROF_STEPS:-200} --warmup 20 --no-cpu-baseline --no-c1 > "$O/profc2.json" 2> "$O/profc2.err") \
        || { tail -20 "$O/profc2.err"; exit 1; }
      python3 tools/trace_step.py "$O/profc2/run_kernel_trace.csv" > "$O/step_c2.txt" || exit 1
      rm -f "$O/profc2/run_kernel_trace.csv"; tail -25 "$O/step_c2.txt" ;;
    ab)
      timeout -k 10 400 python -u tools/ab_bench.py ${AB_ARGS:-} --variants ${AB_VARIANTS:?AB_VARIANTS} \
        > "$O/ab${AB_TAG:-}.txt" 2>&1 || { tail -20 "$O/ab${AB_TAG:-}.txt"; exit 1; }
      cat "$O/ab${AB_TAG:-}.txt" ;;
    parity)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "${PARITY_K:-factorize_matches or full_size or hmc_sweep_matches}" \
        --timeout 300 --timeout-method thread > "$O/parity.log" 2>&1 || { tail -40 "$O/parity.log"; exit 1; }
      tail -3 "$O/parity.log" ;;
    tpar)
      timeout -k 10 600 python -u -m pytest tests/test_transport.py tests/test_gpu_parity.py tests/test_simulation.py -m gpu -x -q \
        -k "${TPAR_K:-eig or transport or eigensystem or measure}" --timeout 300 --timeout-method thread > "$O/tpar.log" 2>&1 \
        || { tail -40 "$O/tpar.log"; exit 1; }
      tail -3 "$O/tpar.log" ;;
    tprof)
      (export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/tprof" -o run -- \
        python3 tools/transport_single.py 32 ${TP_K:-3} ${TP_S:-16} > "$O/tprof.txt" 2> "$O/tprof.err") \
        || { tail -20 "$O/tprof.err"; exit 1; }
      rm -f "$O/tprof/run_kernel_trace.csv"; cat "$O/tprof.txt" ;;
    trans)
      timeout -k 10 200 python -u tests/bench_transport.py --steps 3 --snapshots 4,8,16 > "$O/transport.json" \
        2> "$O/transport.err" || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
