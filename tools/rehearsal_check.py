"""Compare bench lines of a one-rank run and an N-rank run over the same global chains:
python tools/rehearsal_check.py N1.json N2.json [N1b.json N2b.json ...] (pairs).  The reduced
full-diagnostics fields (per configuration) must have identical checksums and the
|cut| histogram mass must equal the yields; prints one verdict line per pair, exits 1 on a
mismatch."""
import json
import sys


def load(path):
    with open(path) as f:
        lines = [ln for ln in f if ln.startswith("{")]
    return json.loads(lines[-1])


def main(paths):
    bad = 0
    for a, b in zip(paths[0::2], paths[1::2]):
        x, y = load(a), load(b)
        rx, ry = x["full_diagnostics"]["reduced"], y["full_diagnostics"]["reduced"]
        same = rx["checksums"] == ry["checksums"] and \
            [g["checksums"] for g in rx["per_group"]] == [g["checksums"] for g in ry["per_group"]]
        mass = rx["cut_hist_mass"] == rx["yields"] and ry["cut_hist_mass"] == ry["yields"]
        ok = same and mass and y["n_gpus"] == y["ranks_seen"] and x["config"]["workload"] == y["config"]["workload"]
        bad += not ok
        print(json.dumps({"one_rank": a, "n_rank": b, "n_gpus": [x["n_gpus"], y["n_gpus"]],
                          "ranks_seen": [x.get("ranks_seen"), y.get("ranks_seen")], "launcher": y.get("launcher"),
                          "backend": y.get("backend"), "chains_total": [x["config"]["chains_per_gpu"] * x["n_gpus"],
                                                                         y["config"]["chains_per_gpu"] * y["n_gpus"]],
                          "yields": [rx["yields"], ry["yields"]], "checksums_identical": same,
                          "hist_mass_ok": mass, "per_rank_kernel_ms": y.get("per_rank_kernel_ms"),
                          "value": [x["value"], y["value"]], "ok": ok}))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main(sys.argv[1:])
