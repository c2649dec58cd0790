"""Native callers of libsort.so on the GPU box, outside Python and torch (so
on the image's HIP 7.2 runtime, as C / C++ / cgo callers load it):

- tests/cpp/test_parallel: the reference's TestParallel
  (benchmark/pkg/sort/libsort_test.go:35-87) restated in C++ -- 16
  concurrent providedGpu callers, then 16 gpuPartial callers, each phase
  within 2 s, results checked against std::sort / the stable partition --
  plus gpuDistribSort callers mixed with single-device ones;
- tests/cpp/test_parallel_asan: the same against build_asan/libsort.so,
  whose host code is compiled with AddressSanitizer (-Xarch_host; device
  code untouched): the device pool's concurrent host code under ASan
  against a real GPU (the reference's libsort_test.go:35-87 callers);
- tests/cpp/test_rccl_native: the C engine over RCCL in a torch-free
  process (the image's /opt/rocm RCCL, as C and Go callers load it), every
  piece through RCCL, 2^27 + 12345 and 2^28 keys.

A missing binary fails: __graft_entry__.build() makes all three and they
travel to the GPU box (not in .gpurunignore)."""
import os
import pathlib
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("exe", ["test_parallel", "test_parallel_asan", "test_rccl_native"])
def test_native_parallel_callers(exe):
    path = ROOT / "tests" / "cpp" / exe
    assert path.exists(), "built by __graft_entry__.build() (make -C tests/cpp)"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0")
    r = subprocess.run([str(path)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-5000:]
    assert r.stdout.strip().endswith("OK")
    assert "ERROR: AddressSanitizer" not in r.stderr
