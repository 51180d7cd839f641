"""The reference's array-handler tests over the HBM handlers (tests/cpp/handler_test.cpp), compiled
with g++ and run:

* CPU, restated base: the package's ArrayHandler restatement (itsolv_hbm/array_handler.h) + the HBM
  handlers over the host emulation of the device ABI (oracle/build/libssp_emul.so);
* CPU, REFERENCE base: the same handler classes compiled against the reference's own
  molpro/linalg/array/ArrayHandler.h (itsolv_hbm/reference_handler.h, the drop-in) -- this is the
  compile-and-run proof that ArrayHandlerHbm / ArrayHandlerHbmSparse subclass the reference's
  interface, including lazy_handle() (ArrayHandler.h:436) and fused_dot / fused_axpy (:271-292).
  Skipped where /root/reference is absent (the GPU box); the binary is built in a temporary
  directory and never leaves this container;
* GPU (-m gpu), restated base over libsubspace_hip.so: the lazy register evaluated as one
  gemm_inner / gemm_outer launch on an MI355X, bit-exact where the reference's eager sequence is.
"""
import os
import subprocess
import tempfile

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SAN = os.environ.get("ITSOLV_SAN_FLAGS", "").split()  # tools/asan_cpu.sh: the sanitizer build
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "cpp", "handler_test.cpp")
REF_SRC = "/root/reference/src"
INC = ["-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "iterative-solver_amd", "include")]


def build_and_run(libdir, lib, extra=()):
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "handler_test")
        cmd = ["g++", "-std=c++17", "-O1", "-Wall", *extra, *SAN, *INC, SRC, "-o", exe, "-L" + libdir, "-l" + lib,
               "-Wl,-rpath," + libdir]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-4000:]
        r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK 0 failure(s)" in r.stdout, r.stdout[-4000:] + r.stderr[-2000:]
    return r.stdout


def emul_dir():
    d = os.path.join(ROOT, "oracle", "build")
    if not os.path.exists(os.path.join(d, "libssp_emul.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    return d


def test_handlers_restated_base_emulated_device():
    out = build_and_run(emul_dir(), "ssp_emul")
    assert "base: restated" in out and out.count("PASS ") == 21


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference tree not present")
def test_handlers_on_the_reference_base_emulated_device():
    out = build_and_run(emul_dir(), "ssp_emul", ["-DWITH_REFERENCE_BASE", "-I" + REF_SRC])
    assert "base: reference" in out and out.count("PASS ") == 20


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference tree not present")
def test_reference_handler_header_compiles_standalone():
    # the INTEGRATION.md snippet's header on its own, against the reference's ArrayHandler.h only
    with tempfile.TemporaryDirectory() as d:
        probe = os.path.join(d, "probe.cpp")
        open(probe, "w").write(
            "#include <itsolv_hbm/reference_handler.h>\n"
            "#include <type_traits>\n"
            "using namespace molpro::linalg;\n"
            "static_assert(std::is_base_of_v<array::ArrayHandler<hbm::Vec, hbm::Vec>, hbm::ArrayHandlerHbm>);\n"
            "static_assert(std::is_base_of_v<array::ArrayHandler<hbm::Vec, std::map<size_t, double>>,"
            " hbm::ArrayHandlerHbmSparse>);\n"
            "static_assert(!std::is_abstract_v<hbm::ArrayHandlerHbm> && !std::is_abstract_v<hbm::ArrayHandlerHbmSparse>);\n"
            "int main() { hbm::ArrayHandlerHbm h; return h.counter().dot; }\n")
        r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-I" + REF_SRC, *INC, probe],
                           capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]


@pytest.mark.gpu
def test_handlers_restated_base_on_mi355x():
    out = build_and_run(os.path.join(ROOT, "iterative-solver_amd", "lib"), "subspace_hip")
    assert out.count("PASS ") == 21
