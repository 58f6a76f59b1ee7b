# flash prefill v2: numerics + microbench + PMC of v2
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "prefill or paged" --timeout 120 --timeout-method thread > gpurun_out/pf_tests.log 2>&1 || { tail -30 gpurun_out/pf_tests.log; exit 1; }
tail -1 gpurun_out/pf_tests.log
timeout -k 10 200 python tools/bench_prefill_attn.py > gpurun_out/pf_bench.jsonl 2>gpurun_out/pf_bench.err || { tail gpurun_out/pf_bench.err; exit 1; }
timeout -k 10 200 python tools/bench_prefill_attn.py --seqs 4 --len 4000 >> gpurun_out/pf_bench.jsonl 2>>gpurun_out/pf_bench.err || exit 1
cat gpurun_out/pf_bench.jsonl
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --output-format csv --pmc $P1 -d gpurun_out/pmcv2 -o run -- python3 tools/bench_prefill_attn.py --only v2 --iters 5 > gpurun_out/pmcv2.log 2>&1 || { tail -20 gpurun_out/pmcv2.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmcv2 --kernel flash_prefill
rm -rf gpurun_out/pmcv2
