"""Runs the native C++ unit tests (tests/cpp, SURVEY §4.1 equivalents) and the
ThreadSanitizer build of the concurrency suite."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _make(target):
    subprocess.run(["make", "-C", ROOT, "-j8", target], check=True,
                   stdout=subprocess.DEVNULL)


def _run(binary, *args, env=None):
    p = subprocess.run([os.path.join(ROOT, "build", binary), *args], capture_output=True,
                       text=True, timeout=900, env=env)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-4000:]
    return p


def test_cpp_unittests():
    _make("test-bin")
    out = _run("dmlc_unittest").stdout
    assert " 0 failed" in out


def test_cpp_concurrency_under_tsan():
    _make("tsan")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    p = _run("dmlc_unittest_tsan", "--filter=", env=env)
    assert "ThreadSanitizer" not in p.stderr


@pytest.mark.slow
def test_cpp_unittests_under_asan_ubsan():
    _make("asan")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1")
    p = _run("dmlc_unittest_asan", env=env)
    assert "runtime error" not in p.stderr
