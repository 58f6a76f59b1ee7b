import sys; sys.path.insert(0,'/root/repo/tests'); sys.path.insert(0,'/root/repo')
import multiprocessing as mp, json
import test_custom_ar as t
if __name__ == "__main__":
    ctx = mp.get_context("spawn"); q = ctx.Queue(); port = t._free_port()
    world = 8
    procs = [ctx.Process(target=t._rank_main, args=(r, world, port, q), daemon=True) for r in range(world)]
    [p.start() for p in procs]
    res = {}
    for _ in procs:
        rank, bad, err = q.get(timeout=200)
        res[rank] = (bad, err)
    [p.join(30) for p in procs]
    print(json.dumps({str(k): [str(v[0])[:300], v[1]] for k, v in sorted(res.items())}))
