#!/usr/bin/env python3
"""Build an A/B variant of libfleetplace.so whose per-kernel translation units (Makefile FFD_TUS,
fp_pipe_tus.h) use another LLVM machine scheduler -- the production recipe otherwise (CPU side,
before a gpurun call):

    tools/build_sched_variant.py <suffix> <strategy> [tu ...]
      -> fleetflow_amd/libfleetplace<suffix>.so, objects in fleetflow_amd/csrc/build/v<suffix>/

<strategy>: default, iterative-maxocc, iterative-ilp, iterative-minreg, max-ilp, max-memory-clause, or
"keep" (the Makefile's own).  Without tu names every TU except big / bigp changes.  EXTRA="-D..." in
the environment adds defines to every translation unit."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "fleetflow_amd", "csrc")


def makefile_tus():
    mk = open(os.path.join(CSRC, "Makefile")).read()
    body = re.search(r"FFD_TUS := ((?:.*\\\n)*.*)", mk).group(1).replace("\\\n", " ")
    return [t.split(":") for t in body.split()]


def main():
    suffix, strategy, names = sys.argv[1], sys.argv[2], sys.argv[3:]
    tus = makefile_tus()
    for t in tus:
        if strategy != "keep" and ((names and t[0] in names) or (not names and t[0] not in ("big", "bigp"))):
            t[5] = strategy
    spec = " ".join(":".join(t) for t in tus)
    print(f"libfleetplace{suffix}.so: FFD_TUS = {spec}")
    extra = os.environ.get("EXTRA", "")
    if extra:
        print(f"  EXTRA = {extra}")
    subprocess.run(["make", "-s", "-j8", "-C", CSRC, f"FFD_TUS={spec}", f"BUILD=build/v{suffix}",
                    f"OUT=../libfleetplace{suffix}.so", f"EXTRA={extra}"], check=True)


if __name__ == "__main__":
    main()
