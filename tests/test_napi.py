"""Run the node-side N-API tests (tests/js/napi_test.js) from pytest."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ADDON = os.path.join(ROOT, "node-fhe-accelerate_amd", "build", "fhe_napi.node")
SCRIPT = os.path.join(ROOT, "tests", "js", "napi_test.js")
ENGINE = os.path.join(ROOT, "tests", "js", "engine_test.js")


def _node():
    node = shutil.which("node")
    if not node or not os.path.exists("/usr/include/node/node_api.h"):
        pytest.skip("node / node_api.h not available")
    if not os.path.exists(ADDON):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "node-fhe-accelerate_amd"), "napi"])
    return node


def test_napi_cpu_contract():
    node = _node()
    r = subprocess.run([node, SCRIPT, "cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_napi_gpu_golden():
    node = _node()
    r = subprocess.run([node, SCRIPT, "gpu"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr


def test_engine_surface_cpu_contract():
    """FHEEngine surface without a GPU: FHEError codes, parameter sets."""
    node = _node()
    r = subprocess.run([node, ENGINE, "cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_engine_surface_gpu_golden():
    """createEngine -> keys -> encrypt -> multiply -> relinearize -> decrypt and
    the TFHE bootstrap through FHEEngine methods only, vs fhe_engine.json."""
    node = _node()
    r = subprocess.run([node, ENGINE, "gpu"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
