# skinny decode GEMMs at M=64: weights streamed from HBM (rotating > 512 MiB) vs cache-resident
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/bench_skinny_rm.py --ms 64 --impls rowmajor --rounds 2 > gpurun_out/mall.jsonl 2>gpurun_out/mall.err || { tail gpurun_out/mall.err; exit 1; }
timeout -k 10 200 python tools/bench_skinny_rm.py --ms 64 --impls rowmajor --rounds 2 --ncopy 1 >> gpurun_out/mall.jsonl 2>>gpurun_out/mall.err || { tail gpurun_out/mall.err; exit 1; }
timeout -k 10 200 python tools/bench_skinny_rm.py --ms 64 --impls rowmajor --rounds 2 --ncopy 3 --ops qkv,o >> gpurun_out/mall.jsonl 2>>gpurun_out/mall.err || { tail gpurun_out/mall.err; exit 1; }
cat gpurun_out/mall.jsonl
