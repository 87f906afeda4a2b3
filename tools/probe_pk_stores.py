"""measure the store pattern the P_k tile design would produce before building
it.  The design keeps element records in LDS for the rows a spatial tile of elements owns whole
and stores those rows' SELL slots from the tile.  The P_k rows sit colour-major in the SELL
(Morton inside a colour: the multicolour sweeps need it), so a tile's rows are spread over every
colour's chunks.  pnp_probe_slot_stores writes every slot of every owned row once, one thread per
row, with the rows in SELL order (the gather pass's stores today), in tile order (as a tile's
elements reach them), tile by tile in SELL order inside each tile, and in random order, and reports
the time per launch; also how many rows a tile of T elements owns whole.
Context: pore_pnp refined k=3, P3 (or P2), PBOperator Jacobian timed beside it.
usage: python tools/probe_pk_stores.py [degree=3] [refine=3] [tile sizes ...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    refine = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    tiles = [int(a) for a in sys.argv[3:]] or [64, 256, 1024]
    cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(refine)
    ctx = P.Context(mesh, P.Params.from_config(cfg), degree=k)
    ctx.set_operator(P.OP_PB)
    ctx.state_set(np.zeros(ctx.nn))
    ctx.assemble_state(2)
    ctx.timers(enable=True, reset=True)
    ctx.assemble_state(10)
    tm = ctx.timers(enable=False)
    jac_us = tm["assemble_ms"] / tm["assemble_launches"] * 1e3
    for T in tiles:
        r = ctx.probe_slot_stores(T, reps=20)
        out = {"degree": k, "mesh": f"pore_pnp k={refine}", "nodes": ctx.nn,
               "pb_jacobian_us": jac_us, "tile_elems": T, **r}
        for key in ("sell", "tile", "tile_sorted", "random"):
            out[f"gbs_{key}"] = r["slot_bytes"] / (r[f"us_{key}"] * 1e-6) / 1e9
        out["rows_whole_frac"] = r["rows_whole"] / max(1, r["rows"])
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
