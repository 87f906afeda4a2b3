"""Bytes one ILU(0) application of the LDS-staged colour sweeps (k_ilu0_solve_lds, bf16 factors)
reads and writes, from the layout's own counts (pnp_info: live split slots, staged list entries),
against bench.py's stored-format model -- to say what the counted traffic
(profiles/r06/pmc_summary.json) is made of.  Per application (colour 0's forward step runs in the
BiCGSTAB update, outside these launches):
  factors      every live L / U slot's bf16 record (U: the diagonal block too), 14 B for the
               7-value PNP block (16 B before ILU_BF16_B7), plus the diagonal block's lower pair
               read again by each forward launch (4 B per row; 16 B before)
  positions    the 2-B list position of every live off-diagonal slot
  staging      every staged list entry: its 4-B row index and the 24-B record it gathers
  rows         d read (24 B) and y written (24 B) per forward row outside colour 0; y re-read
               (24 B) and v written (24 B) per backward row; the last colour's forward and
               backward share one launch (d in, v out)
One JSON line per config.  usage: python tools/ilu_bytes.py [configs=3,5]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402


def system(c):
    if c == 3:
        cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
        return cfg, P.Mesh.read_gmsh(cfg.meshfile).refine(4)
    cfg = P.read_config(os.path.join(ROOT, "data", "pore_without_dna", "pore.cfg"))
    return cfg, P.Mesh.load(cfg.meshfile, size_scale=0.85).refine(6)


def main():
    configs = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "3,5").split(",")]
    for c in configs:
        cfg, mesh = system(c)
        ctx = P.Context(mesh, P.Params.from_config(cfg))
        ctx.set_operator(P.OP_PNP)
        info = ctx.info()
        ctx.close()
        rows = info["nv_owned"]
        nf = info["nfields"]
        rec = 8 * nf  # one row's record
        # colour sizes are not in pnp_info; colour 0 and the last colour are bounded by the
        # row count, so the row terms are given for "all rows" and noted as an upper bound
        Ls, Us = info["lslots_live"], info["uslots_live"]
        nvb = info["nvb"]
        rec_b = 14 if nvb == 7 else 2 * ((nvb + 7) // 8 * 8)  # bf16 bytes per block
        factors = rec_b * (Ls + Us) + (4 if nvb == 7 else rec_b) * rows
        positions = 2 * (Ls + Us - rows)
        staging = (4 + rec) * (info["lsx_entries"] + info["usx_entries"])
        row_terms = 4 * rec * rows
        vb = 2 * (nvb if nvb == 7 else (nvb + 7) // 8 * 8)
        model = (info["lslots"] + info["uslots"]) * (vb + 4) + 8 * nf * rows + 24 * nf * rows
        out = {"config": c, "rows": rows, "lslots_live": Ls, "uslots_live": Us,
               "lslots_stored": info["lslots"], "uslots_stored": info["uslots"],
               "lsx_entries": info["lsx_entries"], "usx_entries": info["usx_entries"],
               "staged_per_live_slot": (info["lsx_entries"] + info["usx_entries"]) / max(1, Ls + Us - rows),
               "MB": {"factors": factors / 1e6, "positions": positions / 1e6,
                      "staging": staging / 1e6, "rows_upper_bound": row_terms / 1e6,
                      "total_upper_bound": (factors + positions + staging + row_terms) / 1e6,
                      "bench_stored_model": model / 1e6}}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
