"""Host side of the C-ABI under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only).

SURVEY §5 "race detection / sanitizers": the GPU pool offers no device sanitizers, so the
host code of ``relativisticgan_amd/csrc/*.hip`` -- descriptor validation, the GEMM / narrow /
dense planners, workspace, pack and BatchNorm-segment sizing, the ``RGAN_EINVAL`` paths of
every compute entry point -- is rebuilt with ``-fsanitize=address,undefined`` on the host half
only (``-Xarch_host``; the device half is compiled normally and never launched) and driven by
``tests/asan/abi_fuzz.cpp``: ~4 M calls over valid descriptors of every layer family the
planners special-case, the same descriptors with extreme field values, and malformed arguments
to every compute entry point (each must answer RGAN_EINVAL before any launch).  Any sanitizer
report or a refused-too-late call fails the test.

The sanitized objects are cached under ``tests/asan/build`` keyed by a hash of the sources
(the first run compiles ~100 s; later runs only link and fuzz).
"""
import hashlib
import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "relativisticgan_amd", "csrc")
INC = os.path.join(ROOT, "include")
HARNESS = os.path.join(ROOT, "tests", "asan", "abi_fuzz.cpp")
BUILD = os.path.join(ROOT, "tests", "asan", "build")
HIPCC = "/opt/rocm/bin/hipcc"
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
       "-Xarch_host", "-fno-sanitize-recover=undefined", "-Xarch_host", "-g"]


def _digest(paths):
    h = hashlib.sha256()
    for p in sorted(paths):
        h.update(p.encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _build():
    from relativisticgan_amd.build import SOURCES
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + [os.path.join(INC, "rgan.h")]
    os.makedirs(BUILD, exist_ok=True)
    objs, jobs = [], []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(BUILD, f"{src[:-4]}-{_digest([path] + headers)}.o")
        objs.append(obj)
        if not os.path.exists(obj):
            jobs.append([HIPCC, "--offload-arch=gfx950", "-O1", "-std=c++17", "-fPIC", "-I" + INC, *SAN,
                         "-Wno-unused-result", "-c", path, "-o", obj + ".tmp"])
    hobj = os.path.join(BUILD, f"abi_fuzz-{_digest([HARNESS] + headers)}.o")
    if not os.path.exists(hobj):
        jobs.append([CLANG, "-O1", "-g", "-std=c++17", "-I" + INC, "-fsanitize=address", "-fsanitize=undefined",
                     "-fno-sanitize-recover=undefined", "-c", HARNESS, "-o", hobj + ".tmp"])

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(f"{' '.join(cmd)}\n{r.stderr[-4000:]}")
        os.replace(cmd[-1], cmd[-1][:-4])

    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        list(ex.map(run, jobs))
    exe = os.path.join(BUILD, "abi_fuzz")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-fsanitize=address", "-fsanitize=undefined", "-o", exe, hobj,
                    *objs], check=True, capture_output=True)
    return exe


@pytest.mark.skipif(not (os.path.exists(HIPCC) and os.path.exists(CLANG)), reason="needs the ROCm toolchain")
def test_c_abi_host_code_under_asan_ubsan():
    exe = _build()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, "20000"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-6000:]
    assert "abi_fuzz ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]


def teardown_module(_mod):
    # keep only the objects of the current sources (the cache would otherwise grow per edit)
    from relativisticgan_amd.build import SOURCES  # noqa: F401
    if not os.path.isdir(BUILD):
        return
    keep = set()
    for f in sorted(os.listdir(BUILD), key=lambda f: os.path.getmtime(os.path.join(BUILD, f)), reverse=True):
        stem = f.split("-")[0]
        if f.endswith(".o") and stem in keep:
            os.unlink(os.path.join(BUILD, f))
        keep.add(stem)
    shutil.rmtree(os.path.join(BUILD, "tmp"), ignore_errors=True)
