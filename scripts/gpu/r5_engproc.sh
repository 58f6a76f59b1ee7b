# the headline workload with the engine in the server's interpreter vs in a child process behind
# ReplicaRouter (one replica): interleaved, 2 rounds, one GPU
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for m in inproc process; do
    timeout -k 10 400 python -u tools/bench_engine_process.py --mode $m > gpurun_out/ep_${m}_$i.jsonl 2> gpurun_out/ep_${m}_$i.err \
      || { tail -20 gpurun_out/ep_${m}_$i.err; exit 1; }
    cat gpurun_out/ep_${m}_$i.jsonl
  done
done
