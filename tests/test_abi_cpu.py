"""The drop-in boundary without a GPU: libsort.so loads, exports every symbol
include/libsort.h declares, the header compiles as C (cgo, gnu99) and C++,
host-only entry points behave like the reference, and the GPU entry points
fail loudly (no silent CPU fallback)."""
import ctypes
import os
import pathlib
import re
import subprocess
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "libsort.h"
LIB = ROOT / "gpu-radix-sort_amd" / "libsort.so"

REFERENCE_ABI = ["initLibSort", "gpuPartial", "providedGpu", "providedCpu", "populateInput",
                 "gpuPartialProfile", "providedGpuProfile"]


def declared_symbols():
    txt = HEADER.read_text()
    return sorted(set(re.findall(r"LIBSORT_API\s+[\w\s\*]+?\b(\w+)\s*\(", txt)))


def test_header_declares_reference_abi():
    names = declared_symbols()
    for n in REFERENCE_ABI:
        assert n in names


def test_library_exports_every_declared_symbol():
    assert LIB.exists(), "build first (python __graft_entry__.py build)"
    out = subprocess.run(["nm", "-D", "--defined-only", str(LIB)], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    missing = [n for n in declared_symbols() if n not in exported]
    assert not missing, missing
    import pylibsort
    assert sorted(pylibsort.EXPORTED_SYMBOLS) == sorted(declared_symbols())


@pytest.mark.parametrize("lang,flags", [("c", ["-std=gnu99"]), ("c++", ["-std=c++14"])])
def test_header_compiles(tmp_path, lang, flags):
    src = tmp_path / ("t.c" if lang == "c" else "t.cpp")
    src.write_text('#include "libsort.h"\nint main(void){ bool (*f)(uint32_t*, uint32_t*, size_t, '
                   'uint32_t, uint32_t) = gpuPartial; return f == 0; }\n')
    cc = "gcc" if lang == "c" else "g++"
    subprocess.run([cc, *flags, "-Wall", "-Werror", "-fsyntax-only", "-I", str(ROOT / "include"), str(src)],
                   check=True)


def test_header_matches_reference_header_types():
    # same C types as the reference libsort/libsort.h:14-32 (unsigned int* for
    # providedGpu/providedCpu, uint32_t* for the others)
    txt = HEADER.read_text()
    assert re.search(r"bool providedGpu\(unsigned int\* h_in, size_t len\)", txt)
    assert re.search(r"bool providedCpu\(unsigned int\* in, size_t len\)", txt)
    assert re.search(r"bool gpuPartial\(uint32_t\* h_in, uint32_t\* boundaries, size_t h_in_len,\s*"
                     r"uint32_t offset, uint32_t width\)", txt)
    assert re.search(r"void populateInput\(uint32_t\* arr, size_t nelem\)", txt)


def test_populate_input_matches_reference_in_fresh_process(golden):
    g, _ = golden
    code = ("import sys; sys.path[:0]=[%r]; import pylibsort, numpy as np; "
            "a=np.frombuffer(pylibsort.generateInputs(8),dtype=np.uint32); "
            "b=np.frombuffer(pylibsort.generateInputs(4),dtype=np.uint32); "
            "print(' '.join(format(int(v),'08x') for v in np.concatenate([a,b])))"
            % str(ROOT / "gpu-radix-sort_amd"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True).stdout
    words = out.split()
    assert words[:8] == g["fresh_process_first_words"]
    assert words[8:] == g["next_call_words_after_8"]


def test_provided_cpu_is_std_sort(oracle_mod):
    import pylibsort
    x = oracle_mod.pcg(4099)
    y = x.copy()
    assert pylibsort.lib().providedCpu(y.ctypes.data, y.size) == 1
    np.testing.assert_array_equal(y, np.sort(x))


def test_config0_provided_cpu_pinned(golden):
    """configs[0] exactly (1M uint32 keys through the
    reference's CPU local sort): in a fresh process, the library's own
    populateInput (utils.cu:65-80) fills 2^20 keys and providedCpu
    (invokers.cu:68-71) sorts them; the sha256 prefixes of input and output
    equal the ones the reference itself produced (pcg_golden.json, 1048576)."""
    g, _ = golden
    code = ("import sys, ctypes, hashlib; sys.path[:0]=[%r]; import pylibsort, numpy as np; "
            "L=pylibsort.lib(); x=np.empty(1<<20, dtype=np.uint32); "
            "L.populateInput(x.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.c_size_t(x.size)); "
            "a=hashlib.sha256(x.tobytes()).hexdigest()[:16]; "
            "assert L.providedCpu(x.ctypes.data_as(ctypes.POINTER(ctypes.c_uint)), ctypes.c_size_t(x.size)) == 1; "
            "print(a, hashlib.sha256(x.tobytes()).hexdigest()[:16])" % str(ROOT / "gpu-radix-sort_amd"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True).stdout.split()
    want = g["sha256_prefix"][str(1 << 20)]
    assert out == [want["input"], want["sorted"]], (out, want)
    assert want["sorted"] == "cfe37c8a9aed0838"


def test_gpu_entry_points_fail_loudly_without_device(capfd):
    import pylibsort
    if pylibsort.gpu_ready():
        pytest.skip("a GPU is present")
    L = pylibsort.lib()
    x = np.arange(100, dtype=np.uint32)[::-1].copy()
    assert L.providedGpu(x.ctypes.data, x.size) == 0
    b = (ctypes.c_uint32 * 256)()
    assert L.gpuPartial(x.ctypes.data, ctypes.addressof(b), x.size, 0, 8) == 0
    assert "initLibSort" in pylibsort.last_error()
    with pytest.raises(RuntimeError):
        pylibsort.sortFull(bytearray(x.tobytes()))
    np.testing.assert_array_equal(x, np.arange(100, dtype=np.uint32)[::-1])  # untouched


def test_ctypes_default_int_restype_sees_false():
    # reference callers (faasTest/pylibsort/sort.py:101) never set restype:
    # the bool return must be readable as a full int
    L = ctypes.CDLL(str(LIB))
    x = np.arange(4, dtype=np.uint32)
    r = L.providedGpu(ctypes.c_void_p(x.ctypes.data), ctypes.c_size_t(4))
    assert r in (0, 1)


def bool_declared_symbols():
    return sorted(set(re.findall(r"LIBSORT_API\s+bool\s+(\w+)\s*\(", HEADER.read_text())))


def test_bool_exports_define_eax():
    """libsort.h declares the reference entry points `bool`
    (libsort/libsort.h:14-32), but ctypes callers with the default restype
    (faasTest/pylibsort/sort.py:101,118) read the whole of eax, and a C++
    `bool` return defines only al.  Every bool export must therefore be an
    alias of the int-returning <name>_impl (libsort_abi.cpp LS_BOOL_ENTRY):
    same address in the symbol table, and the code writes 32-bit eax (no
    `mov ..., %al` / `set.. %al` as the last write before a ret)."""
    out = subprocess.run(["nm", "--defined-only", str(LIB)], capture_output=True, text=True, check=True).stdout
    addr = {}
    for ln in out.splitlines():
        parts = ln.split()
        if len(parts) == 3:
            addr.setdefault(parts[2], parts[0])
    names = bool_declared_symbols()
    assert len(names) >= 30
    for n in names:
        assert n in addr and n + "_impl" in addr, n
        assert addr[n] == addr[n + "_impl"], "%s is not an alias of %s_impl" % (n, n)
    # the exported dynamic symbols do not include the _impl names
    dyn = subprocess.run(["nm", "-D", "--defined-only", str(LIB)], capture_output=True, text=True,
                         check=True).stdout
    assert "_impl" not in dyn
    # machine code of a leaf entry point: returns with a 32-bit write of eax
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if os.path.exists(objdump):
        dis = subprocess.run([objdump, "-d", "--no-show-raw-insn", "--disassemble-symbols=providedCpu_impl",
                              str(LIB)], capture_output=True, text=True, check=True).stdout
        lines = [ln for ln in dis.splitlines() if "\t" in ln]
        rets = [i for i, ln in enumerate(lines) if ln.strip().endswith("retq")]
        assert rets
        for i in rets:
            last_write = next((ln for ln in reversed(lines[:i]) if re.search(r"%(e?ax|al)\b", ln)), "")
            assert "%eax" in last_write or "%rax" in last_write, last_write


def test_tunables_validate():
    import pylibsort
    prev = pylibsort.setDigitBits(4)
    assert pylibsort.getDigitBits() == 4
    pylibsort.setDigitBits(prev)
    with pytest.raises(ValueError):
        pylibsort.setDigitBits(5)
    assert pylibsort.lib().libsortSetAlgorithm(9) == -1
    prev = pylibsort.setAlgorithm("tiles")
    assert pylibsort.setAlgorithm(prev) == "tiles"
    # the multi-GPU stage trace switch (no device needed)
    L = pylibsort.lib()
    prev = L.libsortSetDistribTrace(1)
    assert L.libsortSetDistribTrace(0) == 1
    assert L.libsortSetDistribTrace(prev) == 0


def test_host_checkers():
    import pylibsort
    x = np.array([5, 1, 4, 4, 2, 0x100], dtype=np.uint32)
    d = np.array(sorted(x, key=lambda v: v & 3), dtype=np.uint32)
    b = [0, 2, 3, 3]  # groups: {4,4,0x100}->0 ... computed below
    cnt = np.bincount(x & 3, minlength=4)
    b = np.concatenate([[0], np.cumsum(cnt)[:-1]]).tolist()
    pylibsort.checkPartial(x.tobytes(), d.tobytes(), b, 0, 2)
    with pytest.raises(pylibsort.sortException):
        pylibsort.checkPartial(x.tobytes(), x.tobytes(), b, 0, 2)
    assert pylibsort.boundariesToCaps([0, 2, 5], 40).tolist() == [8, 12, 20]
    pylibsort.checkOrder(np.sort(x))
    with pytest.raises(pylibsort.sortResultException):
        pylibsort.checkOrder(x)


def test_c_caller_links_against_reference_layout(tmp_path):
    """A C caller built the way the reference's callers are (cgo flags
    `--std=gnu99 -I../../../libsort -L../../../libsort -lsort`,
    benchmark/pkg/sort/libsort.go:11-12) against repo:libsort/ links and runs
    the host-only entry points (populateInput, providedCpu) without a GPU."""
    d = ROOT / "libsort"
    if not (d / "libsort.so").exists():
        subprocess.run(["make", "-C", str(d)], check=True, capture_output=True)
    src = tmp_path / "caller.c"
    src.write_text(
        '#include <stdio.h>\n#include "libsort.h"\n'
        "int main(void){ uint32_t a[8]; populateInput(a, 8);\n"
        "  if (!providedCpu(a, 8)) return 2;\n"
        "  for (int i = 1; i < 8; ++i) if (a[i-1] > a[i]) return 3;\n"
        "  printf(\"%08x\\n\", a[0]); return 0; }\n")
    exe = tmp_path / "caller"
    subprocess.run(["gcc", "--std=gnu99", "-O2", "-I", str(d), str(src), "-L", str(d), "-lsort",
                    "-Wl,-rpath," + str(d), "-Wl,-rpath-link,/opt/rocm/lib", "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    # smallest of the first 8 reference PCG words (tests/golden/pcg_golden.json)
    assert out.stdout.strip() == "0f55ac5f"


@pytest.mark.parametrize("order", ["pylibsort_first", "torch_first"])
def test_one_hip_runtime_per_process(order):
    """torch bundles its own HIP runtime; pylibsort must bind libsort.so to it
    whichever is imported first (two runtimes in one process leave torch
    without a GPU)."""
    pytest.importorskip("torch")
    first, second = ("pylibsort", "torch") if order == "pylibsort_first" else ("torch", "pylibsort")
    code = ("import sys; sys.path.insert(0, %r); import %s; import %s; "
            "maps = open('/proc/self/maps').read(); "
            "print(len({l.split()[-1] for l in maps.splitlines() if 'libamdhip64' in l}))"
            % (str(ROOT / "gpu-radix-sort_amd"), first, second))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True).stdout
    assert out.split()[-1] == "1"


def test_system_runtime_opt_out():
    """LIBSORT_HIP_RUNTIME=system (a torch-free worker) keeps the image's HIP
    runtime, which moves pageable host buffers faster than torch's."""
    code = ("import sys; sys.path.insert(0, %r); import pylibsort; "
            "maps = open('/proc/self/maps').read(); "
            "print(sorted({l.split()[-1] for l in maps.splitlines() if 'libamdhip64' in l}))"
            % str(ROOT / "gpu-radix-sort_amd"))
    env = dict(os.environ, LIBSORT_HIP_RUNTIME="system")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True,
                         env=env).stdout
    libs = eval(out.strip().splitlines()[-1])
    assert len(libs) == 1 and "torch" not in libs[0]
