"""pytest configuration: registers the ``gpu`` marker and makes sure the native artefacts exist.

-m "not gpu" tests run here (no GPU): oracle vs known answers and goldens, the builder
restatement, the host logic, and that the C-ABI libraries load and export every symbol the
headers declare. -m gpu tests are the parity tests proper (GPU vs oracle through the C ABI).
"""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "truetrace-unity-pathtracer_amd", "python"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    libs = [os.path.join(REPO, "truetrace-unity-pathtracer_amd", "lib", "libtruetrace_hip.so"),
            os.path.join(REPO, "truetrace-unity-pathtracer_amd", "lib", "libtruetrace_scene.so"),
            os.path.join(REPO, "oracle", "libtt_oracle.so")]
    if not all(os.path.exists(p) for p in libs):
        subprocess.run([sys.executable, "-c", "import __graft_entry__ as g; g.build()"], cwd=REPO, check=True)


@pytest.fixture(scope="session")
def engine():
    import tthip

    if tthip.device_count() == 0:
        pytest.skip("no GPU visible")
    eng = tthip.Engine(0)
    yield eng
    eng.close()
