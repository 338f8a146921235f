#!/bin/bash
# Round-4 GPU passes: bash tools/gpu_r04.sh TAG step [step ...]
#   suite   full `pytest -m gpu` (DWHMC_TSCAN_RECORD -> tscan_record.json)
#   tscan   the published T scan's low-temperature rows (investigation, 8 chains)
#   bench   the driver's command + C3 x200 + C2 + C5
#   prof    rocprofv3 kernel stats + PMC traffic passes (tools/profile_round.sh) + step trace
#   profc2  rocprofv3 kernel stats of the C2 bench (L = 16, beta = 8; PROF_CFG / PROF_STEPS: another config)
#   sq      SQ / MFMA-busy counters of the bench (tools/pmc_sq.sh) + the f64 MFMA peak micro
#   c2rows  C2 with one and two lattice rows per CR block (DWHMC_CR_ROWS), alternated
#   micro   tools/micro/inv16_variants and launch_floor (prebuilt in-tree)
#   tscantest  tests/test_ref_tscan.py on the GPU
#   driver  the driver's bench command only
#   ab      tools/ab_bench.py in-process A/B (AB_VARIANTS, AB_ARGS, AB_TAG)
#   parity  a GPU parity subset (PARITY_K)
#   transab transport timing with DWHMC_EIG_DEFER_MIN = 4 / 1
#   trans   transport timing (single measurement + snapshot batches)
# Every GPU step runs under its own timeout; the first failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    suite)
      DWHMC_TSCAN_RECORD=$O/tscan_record.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
        --timeout 450 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
      tail -3 "$O/tests.log" ;;
    tscan)
      timeout -k 10 600 python -u tools/ref_tscan.py --rows ${TSCAN_ROWS:-6 5 4} --chains ${TSCAN_CHAINS:-8} \
        --extra-eta-mults 1.25 --out "$O/tscan" > "$O/tscan.log" 2>&1 || { tail -20 "$O/tscan.log"; exit 1; }
      tail -5 "$O/tscan.log" ;;
    bench)
      timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.json" 2> "$O/bench_driver.err" \
        || { tail -20 "$O/bench_driver.err"; exit 1; }
      timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-c1 \
        > "$O/bench_C3_200.json" 2> "$O/bench_C3_200.err" || exit 1
      timeout -k 10 300 python -u bench.py --config C2 --steps 200 --warmup 20 --no-cpu-baseline --no-c1 \
        > "$O/bench_C2.json" 2> "$O/bench_C2.err" || exit 1
      timeout -k 10 300 python -u bench.py --config C5 --steps 40 --warmup 8 --no-cpu-baseline --no-c1 \
        > "$O/bench_C5.json" 2> "$O/bench_C5.err" || exit 1
      python - "$O" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "bench_*.json"))):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(os.path.basename(f), round(d["value"], 1), "steps/s", "poles", d["config"]["poles"],
              "frac", round((d.get("roofline") or {}).get("frac") or 0, 3), "alg_frac", d.get("alg_frac_of_peak"))
    except Exception as e:
        print(f, e)
PY
      ;;
    prof)
      bash tools/profile_round.sh "$TAG" r04 || exit 1
      python3 tools/trace_step.py "$R/gpurun_out/prof_$TAG/stats/run_kernel_trace.csv" > "$O/step.txt" || exit 1
      rm -f "$R/gpurun_out/prof_$TAG/stats/run_kernel_trace.csv" ;;
    profc2)
      (export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/profc2" -o run -- \
        python3 bench.py --config ${PROF_CFG:-C2} --steps ${PROF_STEPS:-200} --warmup 20 --no-cpu-baseline --no-c1 > "$O/profc2.json" 2> "$O/profc2.err") \
        || { tail -20 "$O/profc2.err"; exit 1; }
      python3 tools/trace_step.py "$O/profc2/run_kernel_trace.csv" > "$O/step_c2.txt" || exit 1
      rm -f "$O/profc2/run_kernel_trace.csv"; tail -25 "$O/step_c2.txt" ;;
    sq)
      bash tools/pmc_sq.sh "$TAG" || exit 1
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_f64_peak.hip -o "$O/mfma_f64_peak" || exit 1
      timeout -k 10 60 "$O/mfma_f64_peak" > "$O/mfma_f64_peak.txt" 2>&1 || exit 1
      cat "$O/mfma_f64_peak.txt"
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
        SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/peak_pmc" -o run -- "$O/mfma_f64_peak" \
        > "$O/peak_pmc.log" 2>&1) || exit 1
      rm -f "$O/mfma_f64_peak" ;;
    c2rows)
      for r in 1 2 1 2; do
        DWHMC_CR_ROWS=$r timeout -k 10 300 python -u bench.py --config C2 --steps 200 --warmup 20 --no-cpu-baseline \
          --no-c1 > "$O/bench_C2_rows$r.json" 2> "$O/bench_C2_rows$r.err" || exit 1
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), d['config']['poles'], d.get('cr_inv'), d.get('cr_inv_side'))" "$O/bench_C2_rows$r.json"
      done ;;
    micro)
      for m in inv16_variants launch_floor; do
        timeout -k 10 120 tools/micro/$m > "$O/$m.txt" 2>&1 || { cat "$O/$m.txt"; exit 1; }
        cat "$O/$m.txt"
      done ;;
    tscantest)
      DWHMC_TSCAN_RECORD=$O/tscan_record.json timeout -k 10 900 python -u -m pytest tests/test_ref_tscan.py -m gpu -x -q \
        --timeout 600 --timeout-method thread > "$O/tscantest.log" 2>&1 || { tail -40 "$O/tscantest.log"; exit 1; }
      tail -3 "$O/tscantest.log" ;;
    ab)   # AB_VARIANTS / AB_ARGS: tools/ab_bench.py variants and extra arguments (C3 by default)
      timeout -k 10 400 python -u tools/ab_bench.py ${AB_ARGS:-} --variants ${AB_VARIANTS:?AB_VARIANTS} \
        > "$O/ab${AB_TAG:-}.txt" 2>&1 || { tail -20 "$O/ab${AB_TAG:-}.txt"; exit 1; }
      cat "$O/ab${AB_TAG:-}.txt" ;;
    parity)   # a quick GPU parity subset (PARITY_K selects)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "${PARITY_K:-factorize_matches or full_size or hmc_sweep_matches}" \
        --timeout 300 --timeout-method thread > "$O/parity.log" 2>&1 || { tail -40 "$O/parity.log"; exit 1; }
      tail -3 "$O/parity.log" ;;
    driver)
      timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.json" 2> "$O/bench_driver.err" \
        || { tail -20 "$O/bench_driver.err"; exit 1; }
      tail -c 1500 "$O/bench_driver.json" ;;
    transab)   # single-measurement latency: every pass writing (defer from 4 matrices) vs deferred from 1
      for dm in 4 1; do
        DWHMC_EIG_DEFER_MIN=$dm timeout -k 10 300 python -u tests/bench_transport.py --steps 4 --chains 4 --snapshots 16 \
          > "$O/transport_defer$dm.json" 2> "$O/transport_defer$dm.err" || exit 1
        tail -c 600 "$O/transport_defer$dm.json"; echo
      done ;;
    trans)
      timeout -k 10 200 python -u tests/bench_transport.py --steps 3 --snapshots 4,8,16 > "$O/transport.json" \
        2> "$O/transport.err" || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
