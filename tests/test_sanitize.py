"""CPU: the C oracle built with -fsanitize=address,undefined and driven
through every mode it has (oracle/sanitize_main.c) -- memory errors or
undefined behaviour abort the run (sanitizers on host code)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc missing")
def test_oracle_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "orx_san")
    src = os.path.join(ROOT, "oracle")
    subprocess.run(["gcc", "-O1", "-g", "-std=c11", "-Wall", "-Werror",
                    "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-fno-sanitize-recover=all", "-o", exe,
                    os.path.join(src, "sanitize_main.c"), os.path.join(src, "orx_oracle.c")],
                   check=True, capture_output=True, text=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr
    assert r.stdout.count(" ok") == 8, r.stdout
