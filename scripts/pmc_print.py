"""Print derived metrics of scripts/pmc_kernel.sh passes: python scripts/pmc_print.py gpurun_out/pmc_<tag>"""
import collections
import csv
import glob
import re
import sys


def kname(s):
    m = re.search(r"::(\w+)(<[^>]*>)?\(", s)
    return (m.group(1) + (m.group(2) or "")) if m else s[:60]

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = kname(r["Kernel_Name"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
for f in sorted(glob.glob(f"{root}/p1/run_kernel_trace.csv")):
    for r in csv.DictReader(open(f)):
        dur[kname(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, cs in agg.items():
    d = {c: v / cnt[k][c] for c, v in cs.items()}
    g = lambda c: d.get(c, float("nan"))
    us = sum(dur[k]) / max(len(dur[k]), 1) / 1e3
    gui = g("GRBM_GUI_ACTIVE") / 8
    wc = g("SQ_WAVE_CYCLES")
    print(f"== {k}: {us:.1f} us")
    print(f"  MFMA busy {g('SQ_VALU_MFMA_BUSY_CYCLES') / (gui * 1024):.3f}  insts/dispatch MFMA {g('SQ_INSTS_MFMA'):.3g} "
          f"VALU {g('SQ_INSTS_VALU'):.3g} SALU {g('SQ_INSTS_SALU'):.3g} LDS {g('SQ_INSTS_LDS'):.3g} "
          f"VMEM rd {g('SQ_INSTS_VMEM_RD'):.3g} wr {g('SQ_INSTS_VMEM_WR'):.3g}")
    print(f"  wave cycles: wait_any {g('SQ_WAIT_ANY') / wc:.2f} wait_inst {g('SQ_WAIT_INST_ANY') / wc:.2f} "
          f"(lds {g('SQ_WAIT_INST_LDS') / wc:.2f}) active {g('SQ_ACTIVE_INST_ANY') / wc:.2f}; "
          f"LDS bank-conflict/active {g('SQ_LDS_BANK_CONFLICT') / max(g('SQ_LDS_IDX_ACTIVE'), 1):.2f}")
    print(f"  L2 hit {g('TCC_HIT_sum') / (g('TCC_HIT_sum') + g('TCC_MISS_sum')):.2f}  TCP->TCC read req "
          f"{g('TCP_TCC_READ_REQ_sum'):.3g}  FETCH {2 * g('FETCH_SIZE') / 1024:.1f} MB (x2 gfx950 correction)  "
          f"WRITE {g('WRITE_SIZE') / 1024:.1f} MB")
