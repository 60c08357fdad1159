"""The repository lint gate (scripts/lint.py) is part of the CPU suite, as the
reference's `make lint` is part of its CI (scripts/travis/travis_script.sh:4-9)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_lint_clean():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "lint.py")],
                       capture_output=True, text=True)
    assert p.returncode == 0, p.stdout[-4000:]
