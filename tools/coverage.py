"""Line coverage of the native daemon from the C++ unit/stress tests plus the
end-to-end pytest suites (the reference's `make coverage` = go test -coverprofile).

  python tools/coverage.py [--build build/cov] [--out coverage.txt]

Builds an --coverage tree, runs adp_unit_tests, adp_stress, the health model
check (extended alphabet, depth 4) and the CPU pytest suites against it (ADP_BUILD_DIR), then runs gcov on every object of adp_core
and prints per-file and total line coverage of native/src.
"""
import argparse
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(cmd, **kw):
    print("+", " ".join(cmd), flush=True)
    return subprocess.run(cmd, check=True, **kw)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", default=os.path.join(ROOT, "build", "cov"))
    ap.add_argument("--out", default=None)
    ap.add_argument("--skip-tests", action="store_true")
    a = ap.parse_args()
    b = a.build
    if not os.path.exists(os.path.join(b, "CMakeCache.txt")):
        run(["cmake", "-S", os.path.join(ROOT, "native"), "-B", b, "-G", "Ninja", "-DCMAKE_BUILD_TYPE=Debug",
             "-DADP_COVERAGE=ON"], stdout=subprocess.DEVNULL)
    run(["ninja", "-C", b], stdout=subprocess.DEVNULL)
    if not a.skip_tests:
        for gcda in glob.glob(os.path.join(b, "**", "*.gcda"), recursive=True):
            os.unlink(gcda)
        run([os.path.join(b, "adp_unit_tests")], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        run([os.path.join(b, "adp_stress")], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        # the health model check (its workers are forked: their counts merge into the same .gcda files)
        run([os.path.join(b, "adp_health_model"), "--extended", "--depth", "4", "--jobs", "4"],
            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        env = dict(os.environ, ADP_BUILD_DIR=b)
        subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests")], cwd=ROOT, env=env, check=True)
    objdir = os.path.join(b, "CMakeFiles", "adp_core.dir", "src")
    per_file = {}
    for gcno in sorted(glob.glob(os.path.join(objdir, "**", "*.gcno"), recursive=True)):
        r = subprocess.run(["gcov", "-n", "-o", os.path.dirname(gcno), gcno], capture_output=True, text=True,
                           cwd=b)
        for m in re.finditer(r"File '([^']+)'\nLines executed:([\d.]+)% of (\d+)", r.stdout):
            path, pct, n = m.group(1), float(m.group(2)), int(m.group(3))
            if "/native/src/" not in path:
                continue
            rel = path.split("/native/", 1)[1]
            per_file[rel] = (round(pct * n / 100), n)
    lines = [f"{'file':<40} {'lines':>6} {'covered':>8}"]
    tot_c = tot_n = 0
    for f, (c, n) in sorted(per_file.items()):
        lines.append(f"{f:<40} {n:>6} {100.0 * c / n if n else 0:>7.1f}%")
        tot_c += c
        tot_n += n
    lines.append(f"{'TOTAL':<40} {tot_n:>6} {100.0 * tot_c / tot_n if tot_n else 0:>7.1f}%")
    text = "\n".join(lines) + "\n"
    sys.stdout.write(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
