"""Sharded-vs-one-GPU check at size (GPU box): N gloo ranks on the box's one GPU, each drawing and holding only its
slice of a BASELINE config (synth.config_slice), against one context on the whole input (or a golden entry).

    python tools/shard_check.py c4 0.6 2 [--golden c4@1.0/s1_clean] [--no-single] [ENV=VAL ...]

Prints one JSON line: per-rank (CINDs, checksum, join ranges, records, HBM held) and whether the ranks' count and
checksum sum to the reference's.  Library switches (ENV=VAL) apply to the ranks only.
"""
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, cfg, scale, env, q):
    os.environ.update(env)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rdfind_amd import _lib, distributed, synth
    try:
        d, _ = synth.config_slice(cfg, scale, rank, world)
        ms = d.min_support
        with _lib.Context(0) as ctx:
            ctx.set_triples(d.s, d.p, d.o, d.num_terms)
            del d
            t = time.time()
            gs, cs = distributed.run_sharded(ctx, ms, local_slice=True)
            q.put((rank, {"n": ctx.cind_count(), "checksum": ctx.checksum(), "ranges": gs["n_join_ranges"],
                          "records": gs["n_records"], "groups": gs["n_groups"], "light_chunks": cs["n_light_chunks"],
                          "hbm_gib": round(ctx.device_bytes() / 2**30, 1), "s": round(time.time() - t, 2)}))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, f"{type(e).__name__}: {e}"))
    finally:
        dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp
    args = [a for a in sys.argv[1:] if "=" not in a or a.startswith("--")]
    env = dict(a.split("=", 1) for a in sys.argv[1:] if "=" in a and not a.startswith("--"))
    cfg, scale, world = args[0], float(args[1]), int(args[2])
    golden = args[args.index("--golden") + 1] if "--golden" in args else None
    ref = None
    if golden:
        g = json.load(open(os.path.join(ROOT, "tests", "golden", "full_size.json")))[golden]
        ref = {"n": g["n_cinds"], "checksum": int(g["checksum"]), "from": golden}
    elif "--no-single" not in args:
        from rdfind_amd import _lib, synth
        d = synth.config(cfg, scale)
        with _lib.Context(0) as ctx:
            ctx.set_triples(d.s, d.p, d.o, d.num_terms)
            ms = d.min_support
            del d
            ctx.run(ms)
            ref = {"n": ctx.cind_count(), "checksum": ctx.checksum(), "from": "one context",
                   "ranges": ctx.groups["n_join_ranges"]}
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _port()
    procs = [ctxm.Process(target=_rank, args=(r, world, port, cfg, scale, env, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, item = q.get(timeout=900)
        res[r] = item
    for p in procs:
        p.join(timeout=60)
    ok = all(isinstance(v, dict) for v in res.values())
    out = {"config": cfg, "scale": scale, "ranks": world, "env": env, "per_rank": [res[r] for r in range(world)],
           "reference": ref}
    if ok:
        n = sum(res[r]["n"] for r in range(world))
        h = sum(res[r]["checksum"] for r in range(world)) % (1 << 64)
        out["sum"] = {"n": n, "checksum": h}
        out["matches"] = ref is not None and (n, h) == (ref["n"], ref["checksum"])
    print(json.dumps(out), flush=True)
    sys.exit(0 if ok and (out.get("matches", False) or ref is None) else 1)


if __name__ == "__main__":
    main()
