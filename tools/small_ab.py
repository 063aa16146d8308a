#!/usr/bin/env python3
"""Same-box A/B of library builds on uniform small-buffer batches
(measurement tooling): tools/small_batches.py against each build in turn,
ROUNDS times interleaved, each in its own process; one JSON line per
(round, build, length, api) with the build's path added.

    python tools/small_ab.py ROUNDS LEN [LEN ...] LIB [LIB ...]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUN = ("import runpy, sys; sys.path.insert(0, {root!r}); import zipsfs_amd._lib as L; "
       "L.LIB_PATH = {lib!r}; sys.argv = [{script!r}, '10', {lens!r}]; runpy.run_path(sys.argv[0], run_name='__main__')")


def main():
    rounds = int(sys.argv[1])
    lens = ",".join(a for a in sys.argv[2:] if a.isdigit())
    libs = [os.path.abspath(a) for a in sys.argv[2:] if not a.isdigit()]
    for r in range(rounds):
        for lib in libs:
            code = RUN.format(root=ROOT, lib=lib, script=os.path.join(ROOT, "tools", "small_batches.py"), lens=lens)
            p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
            if p.returncode:
                print(p.stderr[-2000:], file=sys.stderr)
                sys.exit(p.returncode)
            for line in p.stdout.splitlines():
                if line.startswith("{"):
                    d = json.loads(line)
                    if d.get("small"):
                        d.update(round=r, lib=os.path.relpath(lib, ROOT))
                        print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
