#!/usr/bin/env python3
"""Clang static analyzer over the native daemon (`make analyze`).

Configures build/analyze with ROCm's clang and a compile database, then runs
every translation unit of native/src, native/mock and native/tools through
`clang++ --analyze` (the default checker set). Prints each warning and a
total; exits 1 if a warning is left that is not in KNOWN.

KNOWN holds the findings read and judged harmless, one (file, checker) each:
  - unix.Stream on `while ((n = fread(...)) > 0)` loops: the checker assumes
    a read after EOF is a mistake; fread() there returns 0 and ends the loop.
  - unix.BlockInCriticalSection in the test mock's event FIFO reader: the
    mock serialises its fake event queue on purpose; it never ships.
"""

import json
import os
import shlex
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "build", "analyze")
CLANG = "/opt/rocm/lib/llvm/bin/clang"
KNOWN = {
    ("native/src/memcap/driver_usage.cc", "unix.Stream"),
    ("native/src/daemon/supervisor.cc", "unix.Stream"),
    ("native/mock/amdsmi_mock.cc", "unix.BlockInCriticalSection"),
}


def units():
    subprocess.run(["cmake", "-S", os.path.join(ROOT, "native"), "-B", BUILD, "-G", "Ninja",
                    "-DCMAKE_BUILD_TYPE=Debug", "-DCMAKE_EXPORT_COMPILE_COMMANDS=ON",
                    f"-DCMAKE_CXX_COMPILER={CLANG}++", f"-DCMAKE_C_COMPILER={CLANG}"],
                   check=True, stdout=subprocess.DEVNULL)
    for e in json.load(open(os.path.join(BUILD, "compile_commands.json"))):
        rel = os.path.relpath(e["file"], ROOT)
        if not rel.startswith(("native/src/", "native/mock/", "native/tools/")):
            continue
        args, skip = [], False
        for a in shlex.split(e["command"]):
            if skip:
                skip = False
            elif a == "-o":
                skip = True
            elif a != "-c":
                args.append(a)
        yield rel, args + ["--analyze", "-Xanalyzer", "-analyzer-output=text", "-o", "/dev/null"], e["directory"]


def run(unit):
    rel, args, cwd = unit
    r = subprocess.run(args, cwd=cwd, capture_output=True, text=True)
    return rel, r.returncode, [ln for ln in r.stderr.splitlines() if ": warning: " in ln]


def main():
    todo = list(units())
    total, unknown = 0, 0
    with ThreadPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        for rel, rc, warns in ex.map(run, todo):
            if rc:
                print(f"{rel}: analyzer exited {rc}")
                unknown += 1
            for w in warns:
                checker = w.rsplit("[", 1)[-1].rstrip("]")
                known = (rel, checker) in KNOWN
                total += 1
                unknown += not known
                print(("known   " if known else "FINDING ") + os.path.relpath(w.split(": warning: ")[0], ROOT)
                      + ": " + w.split(": warning: ", 1)[1])
    print(f"{len(todo)} translation units, {total} warnings, {unknown} not known")
    return 1 if unknown else 0


if __name__ == "__main__":
    sys.exit(main())
