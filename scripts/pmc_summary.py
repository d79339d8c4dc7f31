"""Summarises rocprofv3 PMC sqlite outputs under a directory: counter totals per kernel."""
import glob
import sqlite3
import sys


def main(root):
    for db in sorted(glob.glob(root + "/**/*.db", recursive=True)):
        c = sqlite3.connect(db)
        t = {r[0].split("_0000")[0]: r[0] for r in c.execute("select name from sqlite_master where type='table'")}
        if "rocpd_pmc_event" not in t:
            continue
        q = ("select i.name, sum(e.value) from {e} e join {i} i on e.pmc_id=i.id group by i.name"
             .format(e=t["rocpd_pmc_event"], i=t["rocpd_info_pmc"]))
        print(db)
        for name, v in c.execute(q).fetchall():
            print("  %-24s %16.0f" % (name, v))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
