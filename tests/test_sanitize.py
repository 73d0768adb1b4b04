"""ASan + UBSan run of the CPU oracle (sanitizers on the
CPU restatement).  Builds oracle/_san/liboracle_san.so (`make -C oracle
sanitize`) and reruns the oracle's own test modules against it in a child
interpreter with the sanitizer runtimes preloaded; an address error or any
undefined-behaviour report aborts the child (-fno-sanitize-recover)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


def test_oracle_under_asan_ubsan():
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("sanitizer runtimes not installed")
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"])
    env = dict(os.environ)
    env.update(ORACLE_LIB=os.path.join(ROOT, "oracle", "_san", "liboracle_san.so"),
               LD_PRELOAD=f"{asan}:{ubsan}",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_oracle.py"),
                        os.path.join(ROOT, "tests", "test_oracle_cipher.py")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, tail
