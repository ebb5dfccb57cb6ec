"""Summarise rocprofv3 PMC passes (scripts/pmc.sh) into per-kernel derived metrics."""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"


def kname(s):
    m = re.search(r"::(\w+)(<[^>]*>)?\(", s)
    return (m.group(1) + (m.group(2) or "")) if m else s


agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = kname(r["Kernel_Name"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
for r in csv.DictReader(open(f"{root}/p1/run_kernel_trace.csv")):
    dur[kname(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k in agg:
    d = {c: v / cnt[k][c] for c, v in agg[k].items()}
    g = lambda c: d.get(c, float("nan"))
    us = sum(dur[k]) / len(dur[k]) / 1e3
    print(f"== {k}: {us:.1f} us/dispatch (profiled), GRBM clock {g('GRBM_GUI_ACTIVE') / 8 / (us * 1e-6) / 1e9:.2f} GHz")
    print(f"   MFMA busy fraction: {g('SQ_VALU_MFMA_BUSY_CYCLES') / (g('GRBM_GUI_ACTIVE') / 8 * 1024):.3f}")
    tot = g("SQ_WAVE_CYCLES")
    print(f"   wave-cycle split: wait_any {g('SQ_WAIT_ANY') / tot:.2f}  wait_inst {g('SQ_WAIT_INST_ANY') / tot:.2f}  "
          f"active {g('SQ_ACTIVE_INST_ANY') / tot:.2f}")
    print(f"   insts/dispatch: MFMA {g('SQ_INSTS_MFMA'):.3g} VALU {g('SQ_INSTS_VALU'):.3g} LDS {g('SQ_INSTS_LDS'):.3g}; "
          f"LDS bank-conflict/active {g('SQ_LDS_BANK_CONFLICT') / max(g('SQ_LDS_IDX_ACTIVE'), 1):.2f}")
    print(f"   L2 hit {g('TCC_HIT_sum') / (g('TCC_HIT_sum') + g('TCC_MISS_sum')):.2f}; FETCH_SIZE {g('FETCH_SIZE') / 1024:.1f} MB"
          f"; WRITE_SIZE {g('WRITE_SIZE') / 1024:.1f} MB")
    print(f"   SQ_BUSY_CYCLES {g('SQ_BUSY_CYCLES'):.3g}; SALU {g('SQ_INSTS_SALU'):.3g}; VMEM rd {g('SQ_INSTS_VMEM_RD'):.3g} "
          f"wr {g('SQ_INSTS_VMEM_WR'):.3g}; wait_inst_lds/wave-cycles {g('SQ_WAIT_INST_LDS') / tot:.3f}")
