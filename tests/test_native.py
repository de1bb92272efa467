"""Native checks that need a compiler, not a GPU:
  * FastDiv (csrc/tt_fastdiv.h, the magic-number division of the trace kernel's refill and pixel
    decode) against '/' over every divisor 1..4096, powers of two +-1, divisors near 2^32 and edge /
    random numerators;
  * the CPU oracle built with -fsanitize=address,undefined (SURVEY §5 sanitizers), driven over the
    committed golden scenes through closest-hit, later-bounce, any-hit (all f1 accumulation modes)
    and visibility-check calls in a subprocess that preloads libasan."""
import os
import shutil
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _gxx():
    return shutil.which("g++") and shutil.which("gcc")


@pytest.mark.skipif(not _gxx(), reason="needs g++")
def test_fastdiv_matches_division(tmp_path):
    exe = tmp_path / "test_fastdiv"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), os.path.join(HERE, "native", "test_fastdiv.cpp")],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


@pytest.mark.skipif(not _gxx(), reason="needs gcc")
def test_oracle_under_address_sanitizer(tmp_path):
    so = tmp_path / "libtt_oracle_asan.so"
    subprocess.run(["gcc", "-O1", "-g", "-fPIC", "-std=c11", "-ffp-contract=off", "-fno-omit-frame-pointer",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-shared", "-o", str(so),
                    os.path.join(REPO, "oracle", "tt_oracle.c"), "-lm", "-lpthread"], check=True)
    libasan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    libubsan = subprocess.run(["gcc", "-print-file-name=libubsan.so"], capture_output=True, text=True).stdout.strip()
    env = dict(os.environ, TT_ORACLE_LIB=str(so), LD_PRELOAD=f"{libasan}:{libubsan}",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([sys.executable, os.path.join(HERE, "native", "asan_oracle_driver.py")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "asan oracle ok" in r.stdout, (r.stdout[-2000:] + r.stderr[-4000:])
