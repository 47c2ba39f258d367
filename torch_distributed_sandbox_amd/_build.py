"""In-tree native build for gfx950 (MI355X).

Builds ``torch_distributed_sandbox_amd/_C.so`` from ``csrc/``:

* ``csrc/kernels/*.hip`` — pure HIP/CDNA4 device code (no torch headers, so they
  compile in seconds) with ``extern "C"``-style host launchers declared in
  ``csrc/kernels/launchers.h``;
* ``csrc/*.cpp`` / ``csrc/comm/*.cpp`` — host C++ (torch op registration via
  ``TORCH_LIBRARY``, the TCP store, the host ring backend, the RCCL
  communicator and the gradient-bucket reducer).

We drive ``hipcc --offload-arch=gfx950`` directly through a generated
``build.ninja`` instead of ``torch.utils.cpp_extension.CUDAExtension``: that
path runs hipify over the sources, and this tree is written for CDNA4 only
(no CUDA spellings to translate, no dual paths).

The reference has no native code of its own; everything here
replaces native pieces it pulls from PyTorch.

Usage::

    python -m torch_distributed_sandbox_amd._build          # incremental
    python -m torch_distributed_sandbox_amd._build --clean  # from scratch

A/B kernel experiments build side variants with extra defines into ``_C_<name>.so`` (their
own object directory), loaded instead of ``_C.so`` when ``TDS_SO_VARIANT=<name>`` is set::

    python -m torch_distributed_sandbox_amd._build --variant prio -D TDS_B3_MFMA_PRIO=2
"""
from __future__ import annotations

import argparse
import glob
import os
import shlex
import shutil
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD_DIR = os.path.join(os.path.dirname(PKG_DIR), "build", "native")
OUT_SO = os.path.join(PKG_DIR, "_C.so")
ARCH = os.environ.get("TDS_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


# per-file device-compiler flags.  x_autocorr.hip: the SLP vectorizer pairs the 41 shift
# accumulators into v_pk_fma_f32 whose misaligned operand pairs cost ~4 v_mov per FMA pair
# (322 moves against 80 packed FMAs per row); scalar v_fmac needs none.
# conv2_bwd.hip / conv2_fwd2.hip: packed f32 VALU (the vectorizer's v_pk_fma/add/mul_f32 in the
# staging and epilogue math) costs more issue cycles than scalar ops beside the MFMAs of the
# same SIMD; same-box A/B (tools/gpu_sessions/r3_s14.sh): conv2 backward 1.247 -> 1.109 ms,
# forward 0.621 -> 0.588 ms, bench 3.327 -> 3.112 ms/step.  (convnet_fused.hip keeps it: its
# layer-1 backward ran 0.31 -> 0.36 ms without.)
HIP_FILE_FLAGS = {
    # MFMA results straight into VGPRs: the layer-1 epilogues read every accumulator back
    # (v_accvgpr_read_b32 x 64 per tile and wave with the default AGPR form)
    "convnet_fused.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"],
    "x_autocorr.hip": ["-fno-slp-vectorize"],
    "conv2_bwd.hip": ["-fno-slp-vectorize"],
    "conv2_fwd2.hip": ["-fno-slp-vectorize"],
}
# A/B builds: TDS_NOSLP_FILES=a.hip,b.hip adds -fno-slp-vectorize to those files as well
for _f in filter(None, os.environ.get("TDS_NOSLP_FILES", "").split(",")):
    HIP_FILE_FLAGS.setdefault(_f, []).append("-fno-slp-vectorize")


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce

    torch_dir = os.path.dirname(torch.__file__)
    incs = [
        os.path.join(torch_dir, "include"),
        os.path.join(torch_dir, "include", "torch", "csrc", "api", "include"),
    ]
    libdir = os.path.join(torch_dir, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    del ce
    return incs, libdir, abi


def _ninja_escape(p: str) -> str:
    return p.replace("$", "$$").replace(" ", "$ ").replace(":", "$:")


def _paths(variant: str | None):
    if not variant:
        return BUILD_DIR, OUT_SO
    return BUILD_DIR + "_" + variant, os.path.join(PKG_DIR, f"_C_{variant}.so")


def write_ninja(debug: bool = False, host_sanitize: bool = False, variant: str | None = None,
                defines=()) -> str:
    build_dir, out_so = _paths(variant)
    incs, libdir, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    opt = "-O0 -g" if debug else "-O3"
    common = [
        "-fPIC",
        "-std=c++17",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        f"-I{CSRC}",
        f"-I{os.path.join(ROCM, 'include')}",
        "-Wno-unused-result",
        "-Wno-unused-command-line-argument",
    ] + [f"-D{d}" for d in defines]
    # Device code: gfx950 only.  -munsafe-fp-atomics lets float atomicAdd lower
    # to global_atomic_add_f32 (no CAS loop) for the few reductions that use it.
    hip_flags = common + [
        opt,
        f"--offload-arch={ARCH}",
        "-munsafe-fp-atomics",
    ]
    host_flags = common + [opt, f"-I{py_inc}"] + [f"-I{i}" for i in incs] + [
        "-DTORCH_EXTENSION_NAME=_C",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-Wno-deprecated-declarations",
    ]
    if host_sanitize:
        # Sanitizers on host code only (GPU ASan is not available on the pool).
        host_flags += ["-fsanitize=address,undefined", "-fno-omit-frame-pointer"]
    ldflags = [
        "-shared",
        f"--offload-arch={ARCH}",
        f"-L{libdir}",
        f"-Wl,-rpath,{libdir}",
        "-lc10",
        "-lc10_hip",
        "-ltorch",
        "-ltorch_cpu",
        "-ltorch_hip",
        "-ltorch_python",
        "-lamdhip64",
        "-lrccl",
        "-lpthread",
    ]
    if host_sanitize:
        ldflags += ["-fsanitize=address,undefined"]

    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    cpp_srcs = sorted(glob.glob(os.path.join(CSRC, "*.cpp")) + glob.glob(os.path.join(CSRC, "comm", "*.cpp")))
    headers = sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True))

    lines = [
        "ninja_required_version = 1.3",
        f"hipcc = {hipcc}",
        f"hipflags = {' '.join(shlex.quote(f) for f in hip_flags)}",
        f"hostflags = {' '.join(shlex.quote(f) for f in host_flags)}",
        f"ldflags = {' '.join(shlex.quote(f) for f in ldflags)}",
        "rule hip",
        "  command = $hipcc $hipflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIP $in",
        "rule host",
        "  command = $hipcc -x c++ $hostflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule link",
        "  command = $hipcc $in $ldflags -o $out",
        "  description = LINK $out",
    ]
    objs = []
    for s in hip_srcs + cpp_srcs:
        rel = os.path.relpath(s, CSRC).replace(os.sep, "_")
        o = os.path.join(build_dir, rel + ".o")
        rule = "hip" if s.endswith(".hip") else "host"
        lines.append(f"build {_ninja_escape(o)}: {rule} {_ninja_escape(s)}")
        extra = HIP_FILE_FLAGS.get(os.path.basename(s))
        if extra:
            lines.append(f"  hipflags = $hipflags {' '.join(shlex.quote(f) for f in extra)}")
        objs.append(o)
    lines.append(f"build {_ninja_escape(out_so)}: link {' '.join(_ninja_escape(o) for o in objs)}")
    lines.append(f"default {_ninja_escape(out_so)}")
    os.makedirs(build_dir, exist_ok=True)
    path = os.path.join(build_dir, "build.ninja")
    text = "\n".join(lines) + "\n"
    old = open(path).read() if os.path.exists(path) else None
    if old != text:
        with open(path, "w") as f:
            f.write(text)
    del headers
    return path


def build(clean: bool = False, jobs: int | None = None, verbose: bool = False, debug: bool = False,
          host_sanitize: bool = False, variant: str | None = None, defines=()) -> str:
    build_dir, out_so = _paths(variant)
    if clean and os.path.isdir(build_dir):
        shutil.rmtree(build_dir)
    ninja_file = write_ninja(debug=debug, host_sanitize=host_sanitize, variant=variant, defines=defines)
    ninja = shutil.which("ninja") or os.path.join(os.path.dirname(sys.executable), "ninja")
    jobs = jobs or min(16, os.cpu_count() or 4)
    cmd = [ninja, "-f", ninja_file, "-j", str(jobs)]
    if verbose:
        cmd.append("-v")
    subprocess.run(cmd, check=True, cwd=build_dir)
    return out_so


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--host-sanitize", action="store_true",
                    help="ASan+UBSan on host C++ (store/backends); never on device code")
    ap.add_argument("--variant", default=None, help="side build _C_<variant>.so (A/B experiments)")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra define for a variant")
    a = ap.parse_args(argv)
    if a.defines and not a.variant:
        ap.error("-D needs --variant (the default _C.so is always built without extra defines)")
    print(build(a.clean, a.jobs, a.verbose, a.debug, a.host_sanitize, a.variant, a.defines))


if __name__ == "__main__":
    main()
