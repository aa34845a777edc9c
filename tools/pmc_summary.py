"""Per-entry-point HBM traffic per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

    python tools/pmc_summary.py gpurun_out/<tag>_FETCH_SIZE gpurun_out/<tag>_WRITE_SIZE > profiles/pmc_summary.json

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch.  MI355X_MICROARCH.md (HBM [CDNA4]): on gfx950
FETCH_SIZE counts 128-B read requests at 64 B, i.e. half the bytes of coalesced reads, so reads
are doubled here (`read_correction`).  The bench's roofline.traffic is hbm_bytes_per_launch of
the dominant entry point."""
import collections
import csv
import json
import sys

# entry point (bench stage key) -> (kernels one call launches once each: the call count,
#                                  helper kernels the same call also launches)
ENTRY = {
    "dvcp_fps_ws": (["fps_select_kernel", "fps_kernel"], []),
    "dvcp_knn_tiled": (["knn_tiled_query_kernel"], ["knn_tiled_build_kernel"]),
    "dvcp_sa_group_mlp_ws": (["sa_mlp_mfma_kernel", "sa_mlp_kernel"], ["sa_pre_kernel", "sa_order_kernel"]),
    "dvcp_ball_query_ws": (["bq_tiled_kernel", "bq_wave_kernel", "ball_query_kernel"], ["bq_build_kernel"]),
    "dvcp_dfe_tgt": (["dfe_tgt"], []),
    "dvcp_cpg": (["cpg_kernel"], []),
}
READ_CORRECTION = 2.0


def load(d, counter):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if r["Counter_Name"] == counter:
            per[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return per


def main():
    fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    out = {"_note": "bytes per launch of each entry point (sum over the kernels it launches), "
                    f"reads = FETCH_SIZE x {READ_CORRECTION} (gfx950 counts 128-B requests at 64 B), "
                    "writes = WRITE_SIZE; bench.py --inflight 1 --steps 4 --warmup 1"}
    for entry, (main_k, helpers) in ENTRY.items():
        subs = main_k + helpers
        calls = sum(len(v) for k, v in fetch.items() if any(m in k for m in main_k))
        if not calls:
            continue
        rd = sum(sum(v) for k, v in fetch.items() if any(m in k for m in subs))
        wr = sum(sum(v) for k, v in write.items() if any(m in k for m in subs))
        out[entry] = {"calls": calls, "read_bytes_per_launch": READ_CORRECTION * rd / calls,
                      "write_bytes_per_launch": wr / calls,
                      "hbm_bytes_per_launch": READ_CORRECTION * rd / calls + wr / calls}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
