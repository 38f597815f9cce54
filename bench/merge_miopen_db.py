"""Merge MIOpen text find/perf databases written on a GPU box into miopen_db/ (key union)."""
import glob
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DST = os.path.join(ROOT, "miopen_db")


def merge(src_dir):
    n = 0
    for f in glob.glob(os.path.join(src_dir, "**", "*.txt"), recursive=True):
        if not (f.endswith(".udb.txt") or f.endswith(".ufdb.txt")):
            continue
        dst = os.path.join(DST, os.path.basename(f))
        entries = {}
        for path in (dst, f):
            if os.path.exists(path):
                for line in open(path):
                    line = line.rstrip("\n")
                    if "=" in line:
                        k = line.split("=", 1)[0]
                        entries[k] = line
        with open(dst, "w") as out:
            out.write("\n".join(entries[k] for k in sorted(entries)) + "\n")
        n += len(entries)
    for f in glob.glob(os.path.join(src_dir, "**", "*.ukdb"), recursive=True):
        shutil.copy2(f, os.path.join(DST, os.path.basename(f)))
    return n


if __name__ == "__main__":
    for d in sys.argv[1:]:
        print(d, merge(d))
