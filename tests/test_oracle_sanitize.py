"""The C restatement (oracle/oracle_c.c, checker and CPU baseline) under
AddressSanitizer + UndefinedBehaviorSanitizer: oracle/sanitize_driver.c
calls every entry point on small random instances (evaluation, full /
resync / segment-priced SA, batched TSP SA, brute force); any out-of-bounds
access, leak or undefined operation aborts it.  Host code only (GPU
sanitizers are not available on this pool)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE = os.path.join(os.path.dirname(HERE), "oracle")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_c_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "sanitize_driver")
    cmd = ["gcc", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-ffp-contract=off", "-fopenmp",
           os.path.join(ORACLE, "sanitize_driver.c"), os.path.join(ORACLE, "oracle_c.c"),
           "-lm", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1", OMP_NUM_THREADS="2")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sanitize driver: ok" in r.stdout
