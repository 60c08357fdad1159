"""Package import order: a launcher imports no torch / HIP runtime; any path
into the native extension loads torch first (PyTorch-ROCm and libdmlc.so must
share one libamdhip64, or torch sees no GPU)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(code):
    env = dict(os.environ, PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                         timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    return out.stdout.strip()


def test_launcher_imports_no_torch():
    assert _run("import sys, dmlc_core_amd.parallel.launch.submit, dmlc_core_amd.parallel.tracker;"
                "print('torch' in sys.modules)") == "False"


def test_every_path_to_the_extension_loads_torch_first():
    for stmt in ("from dmlc_core_amd.io import GPURecordIO",
                 "from dmlc_core_amd._dmlc import write_synthetic",
                 "from dmlc_core_amd import _dmlc",
                 "import dmlc_core_amd.data"):
        got = _run(f"import sys; {stmt}; m = list(sys.modules);"
                   "print(m.index('torch') < m.index('dmlc_core_amd._dmlc'))")
        assert got == "True", stmt
