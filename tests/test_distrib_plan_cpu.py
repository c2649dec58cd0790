"""The host arithmetic of the single-process multi-GPU sort (csrc/
distrib_plan.h: round plan, exchange pieces, LSD gather tables, equal re-cut)
exercised by a CPU simulation of R ranks (tests/cpp/distrib_sim.cpp) against
the oracle, compiled with AddressSanitizer + UndefinedBehaviorSanitizer (the
host-code sanitizer build SURVEY.md section 5 asks for)."""
import pathlib
import shutil
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def test_distrib_plan_simulation_asan(tmp_path):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = tmp_path / "distrib_sim"
    subprocess.run([gxx, "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-fno-sanitize-recover=undefined", "-I", str(ROOT / "gpu-radix-sort_amd" / "csrc"),
                    str(ROOT / "tests" / "cpp" / "distrib_sim.cpp"), "-o", str(exe)], check=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600,
                       env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0", "PATH": "/usr/bin:/bin"})
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.startswith("OK")
