set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in "8 1" "4 1" "16 1" "32 1" "8 0" "64 1"; do
  set -- $cfg
  K8SLLM_TILE_GM=$1 K8SLLM_TILE_REMAP=$2 timeout -k 10 120 python -u tools/bench_gemm_tile.py --only down,gate_up+swiglu --impl tile --rounds 2 > gpurun_out/gm.jsonl 2>gpurun_out/gm.err || { tail gpurun_out/gm.err; exit 1; }
  echo "GM=$1 remap=$2"; cat gpurun_out/gm.jsonl
done
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
grep -o "TCC_[A-Z_]*\|TCP_[A-Z_]*" gpurun_out/counters.txt | sort -u | head -80 | tr '\n' ' '
