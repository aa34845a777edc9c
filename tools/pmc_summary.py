"""Per-kernel and per-entry-point PMC figures from rocprofv3 --pmc passes.

    python tools/pmc_summary.py gpurun_out/<tag>_* > profiles/pmc_summary.json

Every argument is a rocprofv3 output directory (run_counter_collection.csv); each pass holds some
of these counters (MI355X_MICROARCH.md, rocprofv3 PMC slots: FETCH_SIZE and WRITE_SIZE need
passes of their own):
  * FETCH_SIZE, WRITE_SIZE (KiB per dispatch) -> HBM bytes.  On gfx950 FETCH_SIZE counts 128-B
    read requests at 64 B, i.e. half the bytes of coalesced reads, so reads are doubled
    (`READ_CORRECTION`, MI355X_MICROARCH.md HBM [CDNA4]);
  * MfmaUtil  = sum SQ_VALU_MFMA_BUSY_CYCLES / (max GRBM_GUI_ACTIVE x SIMD_NUM) x 100,
    VALUBusy  = 100 x sum SQ_ACTIVE_INST_VALU / CU_NUM / max GRBM_GUI_ACTIVE,
    VALUUtilization = 100 x SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64)
    (rocprofv3's own derived-counter expressions, `rocprofv3 -L`), plus raw SQ_INSTS_VALU /
    SQ_INSTS_MFMA / SQ_INSTS_VALU_MFMA_MOPS_F32 / SQ_BUSY_CYCLES / SQ_WAVES per dispatch.
Percentages are averaged over a kernel's dispatches weighted by dispatch duration; an entry point's
figure is the duration-weighted average over the main kernels it launches.  The bench reads the
entry-point records (roofline.traffic, roofline.pmc)."""
import collections
import csv
import json
import os
import sys

# entry point (bench stage key) -> (kernels one call launches once each: the call count,
#                                  helper kernels the same call also launches)
ENTRY = {
    "dvcp_fps_ws": (["fps_select_kernel", "fps_kernel", "fps_split_kernel", "fps_dense_kernel"], []),
    "dvcp_fps_parts": (["fps_part_kernel", "fps_select_kernel", "fps_kernel", "fps_split_kernel", "fps_dense_kernel"],
                       []),
    "dvcp_fps_pair": (["fps_pair_kernel"], ["fps_pair_remap_kernel", "fps_select_gated_kernel"]),
    "dvcp_knn_tiled": (["knn_tiled_query_kernel", "knn_sel_query_kernel"],
                       ["knn_tiled_build_kernel", "knn_qbox_kernel", "knn_qhist_kernel", "knn_qscan_kernel"]),
    "dvcp_sa_group_mlp_ws": (["sa3_mfma_kernel<", "sa_mlp_mfma_kernel<float, 32,"], ["sa_pre_mfma_kernel<32,", "sa_order_kernel"]),
    "dvcp_sa_group_mlp_rows_ws": (["sa_mlp_mfma_kernel<float, 64,"], ["sa_pre_mfma_kernel<64,"]),
    "dvcp_ball_query_ws": (["bq_tiled_kernel", "bq_wave_kernel", "ball_query_kernel"], ["bq_build_kernel", "bq_pack_kernel"]),
    "dvcp_dfe_tgt": (["dfe_tgt"], ["points_pack4_kernel"]),
    "dvcp_cpg": (["cpg_kernel"], []),
}
READ_CORRECTION = 2.0
PCT = ("MfmaUtil", "VALUBusy", "VALUUtilization")
RAW = ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_VALU_MFMA_MOPS_F32", "SQ_BUSY_CYCLES", "SQ_WAVES",
       "GRBM_GUI_ACTIVE")


def short(name):
    n = name.replace("void ", "")
    return n.split("(")[0] if "(" in n else n


def load(dirs):
    """{kernel: {counter: [(value, duration_ns), ...]}}"""
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            dur = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            per[short(r["Kernel_Name"])][r["Counter_Name"]].append((float(r["Counter_Value"]), dur))
    return per


def kernel_record(c):
    rec = {}
    if "FETCH_SIZE" in c:
        rec["calls"] = len(c["FETCH_SIZE"])
        rec["read_bytes_per_launch"] = READ_CORRECTION * 1024.0 * sum(v for v, _ in c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
    if "WRITE_SIZE" in c:
        rec["write_bytes_per_launch"] = 1024.0 * sum(v for v, _ in c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
    for k in PCT:
        if k in c:
            w = sum(d for _, d in c[k]) or 1.0
            rec[k] = sum(v * d for v, d in c[k]) / w
            rec.setdefault("pmc_calls", len(c[k]))
            rec.setdefault("avg_dispatch_us_profiled", w / len(c[k]) / 1e3)
    for k in RAW:
        if k in c:
            rec[k + "_per_launch"] = sum(v for v, _ in c[k]) / len(c[k])
    return rec


def main():
    per = load(sys.argv[1:])
    kernels = {k: kernel_record(c) for k, c in per.items()}
    out = {"_note": "per entry point: HBM bytes per launch (reads = FETCH_SIZE x 2.0, gfx950 counts 128-B "
                    "requests at 64 B; writes = WRITE_SIZE) summed over the kernels it launches, and "
                    "duration-weighted MfmaUtil / VALUBusy / VALUUtilization (%) of its main kernels "
                    "(rocprofv3 derived-counter expressions); bench.py --inflight 1; `kernels` holds "
                    "every kernel's own record"}
    for entry, (main_k, helpers) in ENTRY.items():
        subs = main_k + helpers
        mk = [k for k in kernels if any(m in k for m in main_k)]
        hk = [k for k in kernels if any(m in k for m in subs)]
        if not mk:
            continue
        e = {}
        calls = sum(kernels[k].get("calls", 0) for k in mk)
        if calls:
            rd = sum(kernels[k].get("read_bytes_per_launch", 0) * kernels[k].get("calls", 0) for k in hk)
            wr = sum(kernels[k].get("write_bytes_per_launch", 0) * kernels[k].get("calls", 0) for k in hk)
            e.update(calls=calls, read_bytes_per_launch=rd / calls, write_bytes_per_launch=wr / calls,
                     hbm_bytes_per_launch=(rd + wr) / calls)
        for pk, ok in (("MfmaUtil", "mfma_util"), ("VALUBusy", "valu_busy"), ("VALUUtilization", "valu_util_lanes")):
            ws = [(kernels[k][pk], kernels[k]["avg_dispatch_us_profiled"] * kernels[k]["pmc_calls"])
                  for k in mk if pk in kernels[k]]
            if ws:
                tot = sum(w for _, w in ws) or 1.0
                e[ok] = round(sum(v * w for v, w in ws) / tot, 3)
        if e:
            e["main_kernels"] = mk
            out[entry] = e
    out["kernels"] = kernels
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
