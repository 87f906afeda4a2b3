"""The library's own multi-rank solve across OS processes, on the GPU.

Two processes, each one rank with the host-staged transport (pnp_comm.host: the halo exchange and
every reduction through gloo from Python, staged in pinned host memory), share the box's one
MI355X -- RCCL refuses two ranks on one device, so this is how the library's partitioned BiCGSTAB,
halo exchange, owner-masked dots and Newton run end to end across processes here.  They run the
reference driver's sequence (PB Newton -> BCExtension -> PNP Newton with BiCGSTAB + ILU(0)) on
test/pore_pnp/pore.msh refined twice, and rank 0 compares with a one-rank context:
  * R(x0) of the partitioned assembly: 1e-13 (owner-computes rows, the same element arithmetic);
  * the PB potential (Newton reduction 1e-10) and the PNP solution converged to the rounding floor
    (reduction 1e-13, linear 1e-10): 1e-10 relative -- block-Jacobi ILU(0) across the two ranks is
    a different preconditioner, so only the converged solutions, not the iterates, agree (at the
    reference's Newton reduction 1e-10 they agree to 1.5e-9, round 5 lease h);
  * the ion-current observable at the solution (a boundary flux, differences of the solution):
    1e-8.
The workers are started as child processes (tests/dist_host_worker.py) and bounded by a timeout."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_two_processes_host_transport_match_one_rank(tmp_path):
    port, out = _free_port(), str(tmp_path / "dist_host.json")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_host_worker.py"), str(r),
                               "2", str(port), out], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(2)]
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=150)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    rep = json.load(open(out))
    print(json.dumps(rep))
    assert rep["transport"] == 3 and rep["host_calls_rank0"]["exchange"] > 0, rep
    assert rep["pnp_converged"] == [1, 1], rep
    assert rep["residual_x0_rel_err"] <= 1e-13, rep
    assert rep["phi_pb_rel_err"] <= 1e-10, rep
    assert rep["solution_rel_err"] <= 1e-10, rep
    assert rep["ion_flux_rel_err"] <= 1e-8, rep
