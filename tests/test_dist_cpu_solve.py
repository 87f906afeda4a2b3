"""The multi-rank solve data path over gloo (world_size 2, CPU): each rank takes its RCB
partition and halo plan from the library's host layout (pnp_amd.Layout: owned rows, ghost
columns, per-neighbour send lists), restricts the oracle's PB Jacobian on pore_pnp to its owned
rows over local columns, and runs Jacobi-preconditioned BiCGSTAB with the product's multi-rank
pattern: a halo exchange (isend / irecv of the send lists into the ghost range) before every
SpMV, and owner-masked dots allreduced (the scalar product of ISTL's NOVLP backends,
src/stationary_pnp_from_pb.hh:355-358; pnp_dot / pnp_norm in the library).  The distributed
solution must match a one-process run of the same iteration to 1e-10 and solve the system.
The GPU's RCCL transport needs one GPU per rank; the same plan drives it (ctx.cc)."""
import multiprocessing as mp
import os
import socket

import numpy as np

from conftest import DATA  # noqa: F401  (puts the package on the path)

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def _system():
    import meshio
    import oracle_py as O
    import pnp_amd as P
    z = np.load(os.path.join(GOLD, "pore_pnp_k0.npz"))
    mesh = P.Mesh(z["xy"], z["tri"], z["bseg"], z["bgroup"])
    l_b, c0, tau, cyl, pi = z["params"]
    surfs = [meshio.Surface(int(s[0]), s[1], s[2], int(s[3]), s[4], s[5], int(s[6]), s[7], s[8])
             for s in z["surfaces"]]
    orc = O.Problem(meshio.Mesh(mesh.xy, mesh.tri, mesh.bseg, mesh.bgroup), surfs, l_b=l_b, c0=c0,
                    tau=tau, cylindrical=int(cyl), pi=pi)
    op = orc.operator(O.OP_PB, flux=orc.flux(), mask=orc.mask(1))
    A = orc.jacobian(op, z["pb_x"]).tocsr()
    b = orc.residual(op, z["pb_x"])
    return P, mesh, A, b


def bicgstab_jacobi(matvec, dot, dinv, b, reduction=1e-10, maxit=5000):
    """Textbook BiCGSTAB with a Jacobi preconditioner; matvec / dot hide the distribution."""
    x = np.zeros_like(b)
    r = b.copy()
    rt = r.copy()
    n0 = np.sqrt(dot(r, r))
    rho = alpha = omega = 1.0
    p = np.zeros_like(b)
    v = np.zeros_like(b)
    for it in range(1, maxit + 1):
        rho_new = dot(rt, r)
        beta = (rho_new / rho) * (alpha / omega)
        p = r + beta * (p - omega * v)
        ph = dinv * p
        v = matvec(ph)
        alpha = rho_new / dot(rt, v)
        s = r - alpha * v
        sh = dinv * s
        t = matvec(sh)
        omega = dot(t, s) / dot(t, t)
        x = x + alpha * ph + omega * sh
        r = s - omega * t
        rho = rho_new
        if np.sqrt(dot(r, r)) < reduction * n0:
            return x, it
    return x, maxit


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        P, mesh, A, b = _system()
        L = P.Layout(mesh, rank, world)
        l2g = np.asarray(L.l2g)
        no, nl = int(L.n_owned), len(l2g)
        g2l = np.full(mesh.nv, -1)
        g2l[l2g] = np.arange(nl)
        Ao = A[l2g[:no], :].tocoo()
        cols = g2l[Ao.col]
        assert (cols >= 0).all(), "a coupling outside owned + ghost columns"
        import scipy.sparse as sp
        Al = sp.csr_matrix((Ao.data, (Ao.row, cols)), shape=(no, nl))
        nbrs = [int(p) for p in L.nbr_ranks]
        sidx, sptr, rptr = np.asarray(L.send_idx), np.asarray(L.send_ptr), np.asarray(L.recv_ptr)

        def halo(xo):  # owned values -> local vector with ghosts
            xl = np.zeros(nl)
            xl[:no] = xo
            reqs, bufs = [], []
            for k, p in enumerate(nbrs):
                reqs.append(dist.isend(torch.from_numpy(xl[sidx[sptr[k]:sptr[k + 1]]].copy()), p))
                buf = torch.empty(int(rptr[k + 1] - rptr[k]), dtype=torch.float64)
                reqs.append(dist.irecv(buf, p))
                bufs.append((k, buf))
            for rq in reqs:
                rq.wait()
            for k, buf in bufs:
                xl[no + rptr[k]:no + rptr[k + 1]] = buf.numpy()
            return xl

        def dot(u, w):
            t = torch.tensor([float(np.dot(u, w))], dtype=torch.float64)
            dist.all_reduce(t)
            return float(t[0])

        dinv = 1.0 / A.diagonal()[l2g[:no]]
        x, it = bicgstab_jacobi(lambda u: Al @ halo(u), dot, dinv, b[l2g[:no]])
        out = np.zeros(mesh.nv)
        out[l2g[:no]] = x
        t = torch.from_numpy(out)
        dist.all_reduce(t)
        dist.destroy_process_group()
        q.put((rank, t.numpy(), it, nbrs))
    except Exception as e:  # report to the parent instead of hanging it
        q.put((rank, repr(e), None, None))


def test_two_process_gloo_bicgstab_matches_one_process():
    world = 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda x: x[0])
    for rank, x, it, nbrs in res:
        assert it is not None, x
        assert nbrs == [1 - rank]  # two ranks: each the other's only neighbour
    x2, it2 = res[0][1], res[0][2]
    assert np.array_equal(x2, res[1][1]) and it2 == res[1][2]
    _, _, A, b = _system()
    x1, it1 = bicgstab_jacobi(lambda u: A @ u, np.dot, 1.0 / A.diagonal(), b)
    assert abs(it2 - it1) <= 2, (it1, it2)
    assert np.max(np.abs(x2 - x1)) <= 1e-10 * np.max(np.abs(x1))
    assert np.linalg.norm(A @ x2 - b) <= 1e-9 * np.linalg.norm(b)
