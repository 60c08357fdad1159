"""CPU parser throughput floors (BASELINE config #1 is the CPU path).

Single-thread rows/s through the public Parser<uint32_t>::Create API
(build/dmlc_bench_cpu, the harness shape BASELINE.md's reference numbers
were taken with).  The floors sit well below the measured numbers
(CSV 2.4 M rows/s, LibSVM 0.82 M rows/s on this container vs. the
reference's 1.16-1.64 M and 0.49 M) so they only trip on algorithmic
regressions such as the per-line `reserve` that made CSV quadratic.
"""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN = os.path.join(ROOT, "build", "dmlc_gen")
BENCH = os.path.join(ROOT, "build", "dmlc_bench_cpu")


def _rows_per_sec(uri, fmt):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run([BENCH, uri, fmt, "0", "1", "3"], env=env, check=True,
                         capture_output=True, text=True, timeout=300).stdout
    return json.loads(out.strip().splitlines()[-1])["rows_per_sec"]


@pytest.mark.skipif(not (os.path.exists(GEN) and os.path.exists(BENCH)),
                    reason="native tools not built (make tools)")
@pytest.mark.parametrize("fmt,uri_args,floor", [("csv", "?label_column=0", 0.6e6),
                                                ("libsvm", "", 0.3e6)])
def test_single_thread_parse_floor(tmp_path, fmt, uri_args, floor):
    prefix = str(tmp_path / "d")
    subprocess.run([GEN, fmt, "200000", prefix, "1", "1"], check=True, capture_output=True)
    path = f"{prefix}-0.{fmt}"
    assert os.path.exists(path)
    rps = _rows_per_sec(path + uri_args, fmt)
    assert rps > floor, f"{fmt}: {rps:.0f} rows/s at 1 thread (floor {floor:.0f})"
