#!/usr/bin/env python3
"""Collect the result lines of A/B and ablation logs (gpurun_out/, not
tracked) into profiles/ab_log.md, the committed record that code comments and
DESIGN.md cite as "profiles/ab_log.md (<log name>)".
Usage: python tools/ab_summary.py [--append] <glob> ...
Only measurement lines are kept (tune.py's cand / phases / selection lines,
bench phase lines, pytest summaries)."""
import glob
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "profiles", "ab_log.md")
KEEP = re.compile(r"( cand |phases ms|int8 selection|ms/step|passed|failed|tie-vote parity|"
                  r"rescans=|TF/s|candidate phase|seed)")


def main():
    args = sys.argv[1:]
    append = "--append" in args
    pats = [a for a in args if a != "--append"]
    paths = sorted({p for pat in pats for p in glob.glob(pat)})
    mode = "a" if append and os.path.exists(OUT) else "w"
    with open(OUT, mode) as f:
        if mode == "w":
            f.write("# A/B and ablation record\n\nResult lines of the one-box A/B runs cited in "
                    "code comments and DESIGN.md (full logs stayed in the untracked "
                    "gpurun_out/).  Same-process rows compare; boxes differ by 3-8 %.\n")
        for p in paths:
            lines = [ln.rstrip() for ln in open(p, errors="replace") if KEEP.search(ln)]
            if not lines:
                continue
            f.write("\n## %s\n\n```\n%s\n```\n" % (os.path.basename(p), "\n".join(lines[-40:])))
    print("wrote %s (%d logs)" % (os.path.relpath(OUT, ROOT), len(paths)))


if __name__ == "__main__":
    main()
