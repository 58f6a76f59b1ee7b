# gate_up skinny GEMM workgroup balance probe: N = 24576 / 28672 / 32768 (384 / 448 / 512 workgroups)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_skinny_rm.py --ms 64 --impls rowmajor --ops gate_up_24k,gate_up,gate_up_32k --rounds 3 > gpurun_out/gu_bal.jsonl 2>gpurun_out/gu_bal.err || { tail gpurun_out/gu_bal.err; exit 1; }
cat gpurun_out/gu_bal.jsonl
