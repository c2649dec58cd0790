"""Host code of libsort compiled with AddressSanitizer + UBSan (the
host-code sanitizer build SURVEY.md section 5 asks for) and checked against
the oracle: the single-process multi-GPU sort's arithmetic (csrc/
distrib_plan.h: round plan, exchange pieces, LSD gather tables, equal re-cut)
over a CPU simulation of R ranks (tests/cpp/distrib_sim.cpp), and the
reference-boundaries mode (csrc/boundaries.h, tests/cpp/boundaries_test.cpp)."""
import pathlib
import shutil
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("src", ["distrib_sim", "boundaries_test"])
def test_host_arithmetic_asan(tmp_path, src):
    """distrib_sim: the multi-GPU schedules' host arithmetic over simulated
    ranks; boundaries_test: gpuPartial's reference-boundaries mode
    (csrc/boundaries.h) against oracle_ref_boundaries (sort.cu:367-394)."""
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = tmp_path / src
    subprocess.run([gxx, "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-fno-sanitize-recover=undefined", "-I", str(ROOT / "gpu-radix-sort_amd" / "csrc"),
                    str(ROOT / "tests" / "cpp" / (src + ".cpp")), "-pthread", "-o", str(exe)], check=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600,
                       env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0", "PATH": "/usr/bin:/bin"})
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.startswith("OK")
