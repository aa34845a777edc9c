"""Per-kernel PMC averages from rocprofv3 --pmc output directories (tools/gpu_micro_pmc.sh):
    python tools/micro_pmc.py <dir> [<dir> ...]
Per kernel (averaged over its dispatches): every counter, plus the wave-cycle split
(SQ_WAIT_ANY = parked on s_waitcnt / barrier, SQ_WAIT_INST_ANY = issue-stalled, SQ_ACTIVE_INST_ANY =
issuing; MI355X_MICROARCH.md: the three are disjoint and sum to SQ_WAVE_CYCLES)."""
import collections
import csv
import os
import sys


def main():
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("void ", "").split("(")[0]
            per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, c in sorted(per.items(), key=lambda kv: -max(sum(v) / len(v) for v in kv[1].values())):
        avg = {k: sum(v) / len(v) for k, v in c.items()}
        if avg.get("SQ_WAVE_CYCLES", 0) < 1e6 and avg.get("SQ_BUSY_CYCLES", 0) < 1e5:
            continue
        print(f"== {name}")
        for k in sorted(avg):
            print(f"   {k:28s} {avg[k]:16.1f}")
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            print(f"   split of wave cycles: waiting {avg.get('SQ_WAIT_ANY', 0) / wc:.3f}  issue-stalled "
                  f"{avg.get('SQ_WAIT_INST_ANY', 0) / wc:.3f}  issuing {avg.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f}  "
                  f"(LDS-issue-stalled {avg.get('SQ_WAIT_INST_LDS', 0) / wc:.3f})")
        if "SQ_WAVES" in avg and "SQ_INSTS_LDS" in avg:
            w = avg["SQ_WAVES"]
            print("   per wave: " + "  ".join(f"{k[9:]} {avg[k] / w:.0f}" for k in
                                             ("SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_MFMA",
                                              "SQ_INSTS_VMEM_RD") if k in avg))


if __name__ == "__main__":
    main()
