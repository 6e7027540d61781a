"""Keep profiles/ small: the rows of rocprofv3's per-dispatch CSVs that a
summary is computed from, nothing else.

    python tools/trim_profiles.py [profiles/*.csv ...]     # default: every CSV in profiles/

- `<tag>_pmc_<pass>.csv` (one --pmc pass of the bench command): the timed
  dispatch's rows only -- the last dispatch of the k_render instantiation the
  tag's summary names (`<tag>_summary.json` "kernel"; without a summary, the
  last non-PRIM k_render dispatch).  Everything tools/profile.py derives is
  computed from those rows (summary "counters_timed_dispatch").
- `<tag>_kernel_trace.csv` (--kernel-trace of the same command): the rows of
  the render path's own kernels (k_render, k_primary, k_tile_*), whose
  durations the summaries and DESIGN.md cite; the runtime's copy/fill
  kernels and the scene build's per-level launches are dropped.
- calibration CSVs (`_calib_*`, `_tdcal_pmc`) and `_kernel_stats.csv` are kept
  whole (a few KB each).

tools/profile.py summarize writes the trimmed form directly.
"""
import csv
import glob
import io
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")
RENDER_KERNELS = re.compile(r"k_render|k_primary|k_tile_")
# k_render<MODE, STATS, WIN, PAIR, Q-or-node-format, PRIM, G[, VAR]>: PRIM (the
# primary-hit pass) anchored by position, so a G or VAR argument never reads as it
NON_PRIM = re.compile(r"k_render<-?\d+, (?:false|true), (?:false|true), (?:false|true), (?:false|true|\d+), false, "
                      r"(?:false|true)(?:, \d+)?>")


def _rows(text):
    rd = csv.DictReader(io.StringIO(text))
    return rd.fieldnames, list(rd)


def _write(path, fields, rows):
    buf = io.StringIO()
    w = csv.DictWriter(buf, fieldnames=fields, quoting=csv.QUOTE_NONNUMERIC, lineterminator="\n")
    w.writeheader()
    for r in rows:
        w.writerow(r)
    with open(path, "w") as fh:
        fh.write(buf.getvalue())


def timed_pmc_rows(rows, kernel=None):
    """The rows of the timed dispatch: the last dispatch of `kernel` (exact
    name), or of the last non-PRIM k_render instantiation."""
    if kernel:
        ids = [int(r["Dispatch_Id"]) for r in rows if r["Kernel_Name"] == kernel]
    else:
        ids = [int(r["Dispatch_Id"]) for r in rows if NON_PRIM.search(r["Kernel_Name"])]
    if not ids:
        return []
    last = max(ids)
    return [r for r in rows if int(r["Dispatch_Id"]) == last]


def trim_file(path):
    base = os.path.basename(path)
    m = re.match(r"(.+?)_(pmc_[a-z0-9]+|kernel_trace)\.csv$", base)
    if not m:
        return None
    tag, kind = m.groups()
    text = open(path).read()
    fields, rows = _rows(text)
    if not fields:
        return None
    if kind == "kernel_trace":
        keep = [r for r in rows if RENDER_KERNELS.search(r.get("Kernel_Name", ""))]
    else:
        summ = os.path.join(os.path.dirname(path), tag + "_summary.json")
        if os.path.exists(summ):
            # a summary names the timed kernel: trim to it, or not at all
            try:
                kernel = json.load(open(summ)).get("kernel")
            except ValueError:
                kernel = None
            if not kernel:
                return None
            keep = timed_pmc_rows(rows, kernel)
        else:
            keep = timed_pmc_rows(rows)
        if not keep:
            return None
    if len(keep) == len(rows):
        return 0
    before = len(text)
    _write(path, fields, keep)
    return before - os.path.getsize(path)


def main(paths):
    saved = 0
    for p in paths or sorted(glob.glob(os.path.join(PROF, "*.csv"))):
        s = trim_file(p)
        if s:
            saved += s
    print("trimmed %.1f MB" % (saved / 1e6))


if __name__ == "__main__":
    main(sys.argv[1:])
