#!/bin/bash
# CPU CI (reference: .travis.yml TASK=lint / unittest_gtest, scripts/travis/*.sh):
# lint gate -> native build (host + gfx950 cross-compile) -> C++ unit tests ->
# sanitizer builds of the CPU library (ASan+UBSan, TSan) -> CPU pytest suite.
# GPU tiers (pytest -m gpu, bench.py, rocprofv3) run on an MI355X host:
#   STAGES=test,bench,prof bash scripts/gpu_session.sh
set -euo pipefail
cd "$(dirname "$0")/.."
JOBS="${JOBS:-8}"
python3 scripts/lint.py
make -j"$JOBS" all test-bin tools
build/dmlc_unittest
make -j"$JOBS" asan tsan
build/dmlc_unittest_asan
TSAN_OPTIONS=halt_on_error=1 build/dmlc_unittest_tsan
python3 -m pytest tests -x -q -m "not gpu"
