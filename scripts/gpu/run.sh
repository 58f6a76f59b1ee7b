# Parameterised GPU driver (replaces the one-off scripts/gpu/r2*.sh files).
#
#   gpurun --timeout 1200 -- 'bash scripts/gpu/run.sh suite'
#   gpurun --timeout 900  -- 'bash scripts/gpu/run.sh prof TAG [bench args...]'
#   gpurun --timeout 600  -- 'bash scripts/gpu/run.sh gemm [bench_gemm_tile args...]'
#   gpurun --timeout 600  -- 'bash scripts/gpu/run.sh tests PYTEST_K_EXPR'
#   gpurun --timeout 600  -- 'bash scripts/gpu/run.sh bench TAG [bench args...]'
#   gpurun --timeout 600  -- 'bash scripts/gpu/run.sh pmc TAG COUNTERS -- cmd...'
#   gpurun --timeout 600  -- 'bash scripts/gpu/run.sh tool TAG script.py [args...]'
#   gpurun --timeout 900  -- 'bash scripts/gpu/run.sh rehearse TAG [bench args...]'
#       (a multi-rank bench.py --gpus N on the ONE GPU of the box: every rank on cuda:0, gloo for the
#        host-side groups - exercises the TP / EP / DP code paths; its q/s is not a scaling number)
#
# Serving sweeps are bench runs with different flags, e.g. the mixed prefill budget:
#   run.sh bench mixed16k --steps 4 --warmup 1 --mixed-prefill-tokens 16384
#   run.sh bench pois2k --steps 2 --warmup 1 --mode poisson --rate 12 --batch 64 --mixed-prefill-tokens 2048
#
# Every GPU step has its own time limit and the steps are chained so that the first failure ends
# the call (no retries).  Logs and summaries land in gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
mode=${1:-suite}
shift || true

prof_summary() {  # $1 = rocprofv3 output dir, $2 = tag, $3 = title
  local f
  f=$(find "$1" -name "*results.db" | head -1)
  python3 tools/rocpd_summary.py "$f" --top 40 --title "$3" > "gpurun_out/prof_$2_summary.md"
  python3 tools/rocpd_summary.py "$f" --decode-steps > "gpurun_out/prof_$2_steps.txt" || true
  python3 tools/rocpd_summary.py "$f" --gaps 5.4 >> "gpurun_out/prof_$2_steps.txt" || true
  cat "gpurun_out/prof_$2_steps.txt"
  rm -rf "$1"
}

case "$mode" in
  suite)  # GPU test suite, smoke, headline bench
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
    tail -2 gpurun_out/gputests.log
    timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
    tail -1 gpurun_out/smoke.log
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --out gpurun_out/bench_suite.json \
      > gpurun_out/bench_suite.log 2>&1 || { tail -20 gpurun_out/bench_suite.log; exit 1; }
    cut -c1-300 gpurun_out/bench_suite.json
    ;;
  tests)  # a subset of the GPU tests: run.sh tests 'gemm or skinny'
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$1" \
      > gpurun_out/gputests_k.log 2>&1 || { tail -40 gpurun_out/gputests_k.log; exit 1; }
    tail -3 gpurun_out/gputests_k.log
    ;;
  bench)  # run.sh bench TAG [bench.py args]
    tag=$1; shift
    timeout -k 10 500 python bench.py --out "gpurun_out/bench_$tag.json" "$@" > "gpurun_out/bench_$tag.log" 2>&1 \
      || { tail -20 "gpurun_out/bench_$tag.log"; exit 1; }
    cut -c1-400 "gpurun_out/bench_$tag.json"
    ;;
  prof)  # kernel trace of the headline bench: run.sh prof TAG [bench.py args]
    tag=$1; shift
    root=$PWD
    cd /tmp && export TMPDIR=/tmp && cd "$root"
    timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_$tag" -o run -- \
      python3 bench.py --steps 2 --warmup 1 "$@" > "gpurun_out/prof_$tag.log" 2>&1 \
      || { tail -30 "gpurun_out/prof_$tag.log"; exit 1; }
    tail -1 "gpurun_out/prof_$tag.log" | cut -c1-200
    prof_summary "gpurun_out/prof_$tag" "$tag" "headline bench kernel trace ($tag)"
    ;;
  gemm)  # prefill GEMM microbench: run.sh gemm [--only qkv --impl w4,hipblaslt]
    timeout -k 10 400 python tools/bench_gemm_tile.py "$@" > gpurun_out/gemm.jsonl 2> gpurun_out/gemm.err \
      || { tail -20 gpurun_out/gemm.err; exit 1; }
    cat gpurun_out/gemm.jsonl
    ;;
  tool)  # any tools/*.py microbench: run.sh tool TAG tools/x.py [args]
    tag=$1; shift
    timeout -k 10 400 python "$@" > "gpurun_out/tool_$tag.jsonl" 2> "gpurun_out/tool_$tag.err" \
      || { tail -20 "gpurun_out/tool_$tag.err"; exit 1; }
    cat "gpurun_out/tool_$tag.jsonl"
    ;;
  rehearse)  # run.sh rehearse TAG --gpus 2 --tp 2 --model llama-tiny-d128 ...
    tag=$1; shift
    export K8SLLM_DEVICE=cuda:0 K8SLLM_DIST_BACKEND=gloo
    timeout -k 10 800 python -u bench.py --out "gpurun_out/rh_$tag.json" "$@" > "gpurun_out/rh_$tag.log" 2>&1 \
      || { grep -v Gloo "gpurun_out/rh_$tag.log" | tail -20; exit 1; }
    cut -c1-500 "gpurun_out/rh_$tag.json"
    ;;
  pmc)  # run.sh pmc TAG KERNEL_SUBSTR "PASS1 CTRS" ["PASS2 CTRS" ...] -- python3 tools/x.py args
    tag=$1; kern=$2; shift 2
    passes=()
    while [ $# -gt 0 ] && [ "$1" != "--" ]; do passes+=(--pass "$1"); shift; done
    shift
    root=$PWD
    cd /tmp && export TMPDIR=/tmp && cd "$root"
    python3 tools/gpu_pmc.py "${passes[@]}" --kernel "$kern" --out "gpurun_out/pmc_$tag.jsonl" -- "$@" \
      || { echo "pmc pass failed"; exit 1; }
    cat "gpurun_out/pmc_$tag.jsonl"
    ;;
  *)
    echo "unknown mode $mode"; exit 2 ;;
esac
