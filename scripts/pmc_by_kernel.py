"""Per-kernel summary of rocprofv3 --pmc CSV outputs under a directory: counter averages per
dispatch, plus the usual ratios (VALU / LDS issue share, wait share, LDS bank conflicts)."""
import csv
import glob
import re
import sys
from collections import defaultdict


def main(root):
    per = defaultdict(lambda: defaultdict(dict))  # kernel -> counter -> {(file, dispatch): value}
    import sqlite3
    for fn in glob.glob(root + "/**/*.db", recursive=True):  # rocpd output: kernel dispatch x pmc event
        c = sqlite3.connect(fn)
        q = ("select s.display_name, i.name, d.dispatch_id, e.value from rocpd_pmc_event e "
             "join rocpd_info_pmc i on e.pmc_id = i.id join rocpd_kernel_dispatch d on e.event_id = d.event_id "
             "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
        for name, cn, disp, v in c.execute(q):
            k = re.sub(r"\(.*", "", name).split("::")[-1]
            d = per[k][cn]
            d[(fn, disp)] = d.get((fn, disp), 0.0) + float(v or 0)
    for fn in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                k = re.sub(r"\(.*", "", row.get("Kernel_Name", "")).split("::")[-1]
                c = row.get("Counter_Name")
                key = (fn, row.get("Dispatch_Id"))
                d = per[k][c]
                d[key] = d.get(key, 0.0) + float(row.get("Counter_Value", 0) or 0)
    for k in sorted(per):
        avg = {c: sum(v.values()) / len(v) for c, v in per[k].items()}
        out = ["%s=%.3g" % (c, v) for c, v in sorted(avg.items())]
        wc = avg.get("SQ_WAVE_CYCLES")
        extra = []
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if c in avg:
                    extra.append("%s/wave=%.2f" % (c, avg[c] / wc))
        if "SQ_LDS_BANK_CONFLICT" in avg and avg.get("SQ_LDS_IDX_ACTIVE"):
            extra.append("lds_conflict=%.2f" % (avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"]))
        print(k)
        print("   " + " ".join(out))
        if extra:
            print("   " + " ".join(extra))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
