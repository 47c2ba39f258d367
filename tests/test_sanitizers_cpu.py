"""Host-code sanitizers (SURVEY.md §5 "Race detection / sanitizers").

Builds tests/native/sanitize_host_comm.cpp (the C++ TCP store + host ring backend, one
thread per rank in one process) twice -- AddressSanitizer + UndefinedBehaviorSanitizer, and
ThreadSanitizer (races between the store's server thread, its clients and the ring ranks) --
and runs each at world sizes 2, 3 and 4.  Host code only: GPU ASan is not available here.
libtorch is not instrumented, so the TSan run pins OpenMP to one thread (its thread pool,
used by at::arange & co., would otherwise report races inside libgomp/libtorch).
"""
import os
import shutil
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(HERE, "native", "sanitize_host_comm.cpp")
CSRC = os.path.join(REPO, "torch_distributed_sandbox_amd", "csrc")
OUT_DIR = os.path.join(REPO, "build", "sanitize")
FLAGS = {
    "asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"],
    "tsan": ["-fsanitize=thread"],
}


def _build(kind):
    exe = os.path.join(OUT_DIR, f"{kind}_host_comm")
    sys.path.insert(0, REPO)
    from torch_distributed_sandbox_amd import _build as b

    incs, libdir, abi = b._torch_paths()
    os.makedirs(OUT_DIR, exist_ok=True)
    deps = [SRC] + [os.path.join(CSRC, "comm", f) for f in ("tcp_store.cpp", "host_comm.h", "net.h", "comm.h")]
    if os.path.exists(exe) and os.path.getmtime(exe) > max(os.path.getmtime(d) for d in deps):
        return exe
    cxx = shutil.which("g++") or "c++"
    cmd = [cxx, "-std=c++17", "-O1", "-g", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-I{CSRC}",
           "-Wno-deprecated-declarations"] + FLAGS[kind] + [f"-I{i}" for i in incs] + [
        SRC, "-o", exe, f"-L{libdir}", f"-Wl,-rpath,{libdir}", "-ltorch_cpu", "-lc10", "-ltorch", "-lpthread"]
    subprocess.run(cmd, check=True, timeout=600)
    return exe


@pytest.fixture(scope="module", params=["asan", "tsan"])
def sanitized(request):
    if shutil.which("g++") is None and shutil.which("c++") is None:
        pytest.skip("no host C++ compiler")
    return request.param, _build(request.param)


@pytest.mark.parametrize("world", [2, 3, 4])
def test_host_comm_under_sanitizers(sanitized, world):
    kind, exe = sanitized
    env = dict(os.environ)
    # libtorch itself is not instrumented: skip its ODR / alloc-dealloc noise and leaks of
    # its static registries; everything in our TU is still checked
    env["ASAN_OPTIONS"] = "detect_odr_violation=0:alloc_dealloc_mismatch=0:detect_leaks=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    env["TSAN_OPTIONS"] = "halt_on_error=1"
    if kind == "tsan":
        env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([exe, str(world)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert f"sanitize_host_comm ok: world={world}" in r.stdout
    for marker in ("runtime error", "AddressSanitizer", "ThreadSanitizer"):
        assert marker not in r.stderr, r.stderr[-4000:]


@pytest.mark.parametrize("kind", ["plain", "tsan"])
def test_rccl_settle_abort_protocol(kind):
    """The native RCCL communicator's lock protocol (csrc/comm/settle.h): an abort requested
    while a non-blocking call settles under the communicator lock is honoured within one poll
    (not after the call's 20 s timeout), and the watchdog's poll never blocks behind the call.
    Also built under ThreadSanitizer."""
    if shutil.which("g++") is None and shutil.which("c++") is None:
        pytest.skip("no host C++ compiler")
    os.makedirs(OUT_DIR, exist_ok=True)
    exe = os.path.join(OUT_DIR, f"settle_protocol_{kind}")
    src = os.path.join(HERE, "native", "settle_protocol.cpp")
    cxx = shutil.which("g++") or "c++"
    flags = ["-fsanitize=thread"] if kind == "tsan" else []
    subprocess.run([cxx, "-std=c++17", "-O1", "-g", f"-I{CSRC}"] + flags + [src, "-o", exe, "-lpthread"],
                   check=True, timeout=300)
    p = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "settle protocol ok" in p.stdout
