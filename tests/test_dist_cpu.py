"""bench.py's multi-rank host path in real processes over gloo (world_size 2, CPU): the
weak-scaling mesh, each rank's RCB partition and halo lists (checked for symmetry across the
processes through gloo collectives), and the max-over-ranks timing reduction.  The RCCL data
path itself needs one GPU per rank (RCCL refuses two ranks on one device); its logic runs in
tests/test_gpu_multirank.py through the in-process transport."""
import importlib.util
import multiprocessing as mp
import os
import socket

import numpy as np

from conftest import DATA

ROOT = os.path.dirname(DATA)


def _bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    B = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(B)
    return B


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        B = _bench()
        P = B.P
        base = P.Mesh.read_gmsh(os.path.join(DATA, "pore_pnp", "pore.msh"))
        mesh = B.tile_mesh(base, world)
        L = P.Layout(mesh, rank, world)
        owned = L.l2g[:L.n_owned].tolist()
        recv = {int(p): L.l2g[L.n_owned + L.recv_ptr[k]:L.n_owned + L.recv_ptr[k + 1]].tolist()
                for k, p in enumerate(L.nbr_ranks)}
        send = {int(p): L.l2g[L.send_idx[L.send_ptr[k]:L.send_ptr[k + 1]]].tolist()
                for k, p in enumerate(L.nbr_ranks)}
        everyone = [None] * world
        dist.all_gather_object(everyone, (owned, recv, send, mesh.nv))
        t = B.max_over_ranks(dist, world, float(rank + 1))
        B.barrier_sync(dist, world)
        dist.destroy_process_group()
        q.put((rank, everyone, t))
    except Exception as e:  # report to the parent instead of hanging it
        q.put((rank, repr(e), None))


def test_two_process_gloo_partition_and_halo():
    world = 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda x: x[0])
    for rank, everyone, t in res:
        assert t is not None, everyone
        assert t == float(world)  # max over ranks of (rank + 1)
    everyone = res[0][1]
    assert everyone == res[1][1]
    nv = everyone[0][3]
    owned = sorted(sum((e[0] for e in everyone), []))
    assert owned == list(range(nv))
    for r, (_, recv, _, _) in enumerate(everyone):
        for p, ghosts in recv.items():
            assert everyone[p][2][r] == ghosts  # p sends r exactly r's ghosts, in order
            assert len(ghosts) > 0


def test_guarded_leg_records_an_error_and_passes_results_through():
    """a secondary bench leg that raises on every rank costs the line that leg only"""
    import pnp_amd as P
    B = _bench()
    assert B.guarded(0, "ok", lambda: {"seconds": 1.0}) == {"seconds": 1.0}

    def boom():
        raise P.PnpError(P.E_STATE, "leg failed")
    out = B.guarded(0, "boom", boom)
    assert set(out) == {"error"} and "leg failed" in out["error"]
