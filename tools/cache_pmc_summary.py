"""Summarise tools/gpu_cache_pmc.sh into profiles/<tag>_<workload>_l1l2.json: per launch of the
flip kernel, L1 (TCP) and L2 (TCC) request counts, wave-state cycles, and the roofline split by
level (bench.roofline_levels) -- the LDS-resident state bytes and the global node-record bytes of
SURVEY §8(d)'s algorithmic count, each against its own peak.

    python tools/cache_pmc_summary.py <tag> <workload>
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def counters(d):
    """{counter: mean value per dispatch} over the flip-kernel dispatches of one pass."""
    vals = {}
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for fn in files:
        for r in csv.DictReader(open(fn)):
            name = r["Kernel_Name"]
            if "flip" not in name or "kernel" not in name:
                continue
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main(tag, wl):
    import bench
    src = os.path.join(ROOT, "gpurun_out", f"cache_{tag}_{wl}")
    line = json.loads([ln for ln in open(os.path.join(src, "bench.json")) if ln.startswith("{")][-1])
    c, n = {}, {}
    for i in (1, 2, 3):
        ci, ni = counters(os.path.join(src, f"pmc{i}"))
        c.update(ci)
        n.update(ni)
    rf = line["roofline"]
    t = rf["kernel_ms"] * 1e-3
    W = bench.Workload(wl)
    per_launch_props = line["value"] * line["ms_per_step"] * 1e-3 / line["n_gpus"]
    acc_pp = line["accept_per_proposal"]
    lv = bench.roofline_levels(W, per_launch_props, per_launch_props * acc_pp, rf["kernel_ms"],
                               rf.get("traffic"))
    line_b = 128.0  # gfx950 L1 / L2 cache line (bytes): requests are priced at a full line (upper bound)
    l2_req = c.get("TCC_REQ_sum")
    meas = {
        "tcp_cache_line_accesses": c.get("TCP_TOTAL_CACHE_ACCESSES_sum"),
        "tcp_reads": c.get("TCP_TOTAL_READ_sum"), "tcp_writes": c.get("TCP_TOTAL_WRITE_sum"),
        "tcp_to_tcc_read_requests": c.get("TCP_TCC_READ_REQ_sum"),
        "tcc_requests": l2_req, "tcc_reads": c.get("TCC_READ_sum"),
        "tcc_hit": c.get("TCC_HIT_sum"), "tcc_miss": c.get("TCC_MISS_sum"),
        "tcc_hit_rate": (c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]))
        if c.get("TCC_HIT_sum") is not None and (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]) > 0 else None,
        "l1_hit_rate_est": (1 - c["TCP_TCC_READ_REQ_sum"] / c["TCP_TOTAL_CACHE_ACCESSES_sum"])
        if c.get("TCP_TOTAL_CACHE_ACCESSES_sum") else None,
        "l2_bytes_upper": l2_req * line_b if l2_req is not None else None,
        "l2_gbs_upper": l2_req * line_b / t / 1e9 if l2_req is not None else None,
        "l2_frac_upper": l2_req * line_b / t / 1e9 / bench.L2_PEAK_GBS if l2_req is not None else None,
        "waves": c.get("SQ_WAVES"), "vmem_rd_insts": c.get("SQ_INSTS_VMEM_RD"), "smem_insts": c.get("SQ_INSTS_SMEM"),
        "flat_insts": c.get("SQ_INSTS_FLAT"),
        "wave_cycles": c.get("SQ_WAVE_CYCLES"),
        "wait_any_frac": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else None,
        "wait_inst_any_frac": c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else None,
        "active_inst_any_frac": c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else None,
    }
    # the library's content hash: bench.measured_l2 reports these counters only for the same build
    out = {"tag": tag, "workload": wl, "kernel": rf["kernel"], "build_id": line.get("build_id"),
           "kernel_ms_bench": rf["kernel_ms"],
           "chains": line["config"]["chains_per_gpu"], "chain_steps": line["config"]["chain_steps_per_launch"],
           "proposals_per_launch": per_launch_props, "counters_per_dispatch": c, "dispatches": n,
           "measured": meas, "levels": lv,
           "notes": ["counters are per dispatch of the flip kernel, averaged over the dispatches of each pass",
                     "TCC requests priced at a 128-B line: an upper bound on L2 bytes (requests may be 32 / 64 B)",
                     "levels: SURVEY §8(d) algorithmic bytes split by where they live -- LDS-resident chain state "
                     "(boundary entry, a[v], a[] of neighbours and ring cells, populations; every write) against "
                     "the LDS aggregate at the access-width mix, global node records (row_ptr pair, col_idx, "
                     "ring indices) against the L2 aggregate (MI355X_MICROARCH.md §L2, 34.5 TB/s), measured HBM "
                     "bytes against 8 TB/s"]}
    # beside the raw passes (merged back from the GPU box) and under profiles/ (committed)
    json.dump(out, open(os.path.join(src, "l1l2.json"), "w"), indent=1)
    json.dump(out, open(os.path.join(ROOT, "profiles", f"{tag}_{wl}_l1l2.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
