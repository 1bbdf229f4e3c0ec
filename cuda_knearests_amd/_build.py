"""Native build for gfx950 (no setuptools/hipify in the loop: explicit hipcc command lines).

Artifacts (all in-tree, so they travel to the GPU box with the repo snapshot):

* ``cuda_knearests_amd/_C*.so``            -- PyTorch extension (GPU ops + CPU oracles)
* ``cuda_knearests_amd/lib/libknearests.so`` -- standalone C API (``csrc/include/knearests.h``)
* ``bin/knn_cli``                           -- reference-equivalent driver (test_knearests.cu)
* ``bin/knn_unit``                          -- C++ unit tests (CPU + GPU sections)

Usage: ``python -m cuda_knearests_amd._build [--jobs N] [--force]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "cuda_knearests_amd"
CSRC = ROOT / "csrc"
OBJ = ROOT / "build" / "obj"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")

KERNELS = ["kernels/build.hip", "kernels/query.hip", "kernels/route.hip", "kernels/tree.hip"]
HOST = ["host/host.cpp"]
RUNTIME = ["runtime/engine.cpp", "runtime/api.cpp", "runtime/hostio.cpp", "runtime/pipeline.cpp", "runtime/dist.cpp"]
HIP_TOOLS = ["tools/cu_mask_probe.hip", "tools/repro_capture.hip"]
MULTI = "runtime/multi.cpp"  # C-API multi-GPU runtime: libknearests.so only (links RCCL)
RCCL_OK = os.path.exists(os.path.join(ROCM, "include", "rccl", "rccl.h"))

CXX = os.environ.get("CXX", "g++")
COMMON = ["-O3", "-std=c++17", "-fPIC", f"-I{CSRC / 'include'}", "-D__HIP_PLATFORM_AMD__=1"]
# device code: hipcc for gfx950 only
# -fno-slp-vectorize: the SLP vectorizer packs pairs of scalar f32 sub/mul/fma into v_pk_*_f32,
# which issue in 4 cycles per wave64 instruction on gfx950 where the scalar forms take 2
# (profiles/valu_rate_r3.txt), plus the v_mov pairing: a loss in VALU-bound kernels.
HIPFLAGS = COMMON + [f"--offload-arch={ARCH}", "-x", "hip", "-munsafe-fp-atomics", "-fno-slp-vectorize",
                     "-Wno-unused-result", "-Wno-unused-value"]
# host-only code (runtime, oracles, bindings, tools): the system C++ compiler + HIP headers
HOSTFLAGS = COMMON + [f"-I{ROCM}/include", "-fopenmp", "-Wall", "-Wno-unused-result",
                      "-Wno-unused-variable"]


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def _digest(paths: list[Path], extra: str) -> str:
    h = hashlib.sha1(extra.encode())
    for p in sorted(paths):
        h.update(p.read_bytes())
    return h.hexdigest()


def _headers() -> list[Path]:
    return sorted((CSRC / "include").rglob("*.h")) + sorted(CSRC.rglob("*.hpp"))


def _compile(src: str, flags: list[str], tag: str, force: bool) -> Path:
    s = CSRC / src
    out = OBJ / f"{tag}_{src.replace('/', '_')}.o"
    stamp = out.with_suffix(".sha1")
    dig = _digest([s] + _headers(), " ".join(flags))
    if not force and out.exists() and stamp.exists() and stamp.read_text() == dig:
        return out
    out.parent.mkdir(parents=True, exist_ok=True)
    compiler = HIPCC if src.endswith(".hip") else CXX
    _run([compiler] + flags + ["-c", str(s), "-o", str(out)])
    stamp.write_text(dig)
    return out


def _torch_flags() -> tuple[list[str], list[str], str]:
    import torch
    from torch.utils import cpp_extension as ce

    inc = [f"-I{p}" for p in ce.include_paths(device_type="cuda")]
    inc.append(f"-I{sysconfig.get_paths()['include']}")
    import pybind11

    inc.append(f"-I{pybind11.get_include()}")
    libdirs = ce.library_paths(device_type="cuda")
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    ldflags = [f"-L{d}" for d in libdirs] + [f"-Wl,-rpath,{tlib}",
               "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python"]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    defs = ["-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H", "-DUSE_ROCM=1",
            f"-D_GLIBCXX_USE_CXX11_ABI={abi}"]
    ext = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return inc + defs, ldflags, ext


def build(jobs: int = 8, force: bool = False, verbose: bool = True) -> dict:
    """Compile every native component. Returns a dict of artifact paths."""
    tflags, tld, ext = _torch_flags()
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = {}
        for k in KERNELS:
            futs[ex.submit(_compile, k, HIPFLAGS, "hip", force)] = ("kern", k)
            # bounds-checked variant (KN_CHECKED=1 -> cuda_knearests_amd._C_checked)
            futs[ex.submit(_compile, k, HIPFLAGS + ["-DKN_CHECKED=1"], "hipchk", force)] = ("kernchk", k)
        for h in HOST:
            futs[ex.submit(_compile, h, HOSTFLAGS, "host", force)] = ("host", h)
        for r in RUNTIME:
            futs[ex.submit(_compile, r, HOSTFLAGS, "rt", force)] = ("rt", r)
        futs[ex.submit(_compile, "torch/bindings.cpp", HOSTFLAGS + tflags + ["-Wno-unused-function"],
                       "torch", force)] = ("torch", "bindings")
        chk_tflags = [f for f in tflags if not f.startswith("-DTORCH_EXTENSION_NAME")]
        futs[ex.submit(_compile, "torch/bindings.cpp", HOSTFLAGS + chk_tflags +
                       ["-Wno-unused-function", "-DTORCH_EXTENSION_NAME=_C_checked", "-DKN_CHECKED=1"],
                       "torchchk", force)] = ("torchchk", "bindings")
        futs[ex.submit(_compile, MULTI, HOSTFLAGS + (["-DKN_HAVE_RCCL=1"] if RCCL_OK else []), "rt", force)] = \
            ("multi", MULTI)
        futs[ex.submit(_compile, "tools/knn_cli.cpp", HOSTFLAGS, "tool", force)] = ("tool", "cli")
        futs[ex.submit(_compile, "tools/knn_unit.cpp", HOSTFLAGS, "tool", force)] = ("tool", "unit")
        # standalone HIP diagnostics (no library): CU-mask -> XCD / CU probe, the capture reproducer
        for t in HIP_TOOLS:
            futs[ex.submit(_compile, t, HIPFLAGS, "hiptool", force)] = ("hiptool", t)
        objs: dict[str, list[Path]] = {"kern": [], "kernchk": [], "host": [], "rt": [], "torch": [],
                                       "torchchk": [], "tool": [], "multi": [], "hiptool": []}
        tools: dict[str, Path] = {}
        for f in cf.as_completed(futs):
            kind, name = futs[f]
            o = f.result()
            objs[kind].append(o)
            if kind == "tool":
                tools[name] = o
    kern = sorted(objs["kern"])
    host = sorted(objs["host"])
    rt = sorted(objs["rt"])
    libdir = PKG / "lib"
    libdir.mkdir(exist_ok=True)
    lib = libdir / "libknearests.so"
    hiplink = [f"--offload-arch={ARCH}", "-fopenmp", f"-L{ROCM}/lib", "-lamdhip64"]
    _run([HIPCC, "-shared", "-o", str(lib)] + [str(o) for o in kern + host + rt + objs["multi"]] + hiplink +
         (["-lrccl", f"-Wl,-rpath,{ROCM}/lib"] if RCCL_OK else []))
    cext = PKG / f"_C{ext}"
    # the extension's RCCL is torch's own (same soname, already loaded by libtorch_hip)
    rccl = ["-lrccl"] + [f"-Wl,-rpath,{ROCM}/lib"]
    _run([HIPCC, "-shared", "-o", str(cext)] + [str(o) for o in kern + host + rt + objs["torch"]] + hiplink + tld + rccl)
    cchk = PKG / f"_C_checked{ext}"
    _run([HIPCC, "-shared", "-o", str(cchk)] + [str(o) for o in sorted(objs["kernchk"]) + host + rt + objs["torchchk"]]
         + hiplink + tld + rccl)
    bindir = ROOT / "bin"
    bindir.mkdir(exist_ok=True)
    exes = {}
    for name, o in tools.items():
        exe = bindir / f"knn_{name}"
        _run([HIPCC, "-o", str(exe), str(o), str(lib), f"-Wl,-rpath,{libdir}", f"-Wl,-rpath,$ORIGIN/../cuda_knearests_amd/lib"]
             + hiplink)
        exes[name] = exe
    for o in objs["hiptool"]:
        exe = bindir / o.stem.replace("hiptool_tools_", "").replace(".hip", "")
        _run([HIPCC, "-o", str(exe), str(o)] + hiplink)
        exes[exe.name] = exe
    res = {"ext": cext, "ext_checked": cchk, "lib": lib, **{f"bin_{k}": v for k, v in exes.items()}}
    if verbose:
        for k, v in res.items():
            print(f"[build] {k}: {v}")
    return res


def build_variant(name: str, hip_flags: list[str], jobs: int = 8) -> Path:
    """Extension ``cuda_knearests_amd._C_<name>`` with extra kernel compile flags, for in-process
    A/B timing of kernel variants (scripts/ab_variant.py)."""
    tflags, tld, ext = _torch_flags()
    tag = "var_" + name
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        kf = [ex.submit(_compile, k, HIPFLAGS + hip_flags, tag, False) for k in KERNELS]
        hf = [ex.submit(_compile, h, HOSTFLAGS, "host", False) for h in HOST]
        rf = [ex.submit(_compile, r, HOSTFLAGS, "rt", False) for r in RUNTIME]
        base = [f for f in tflags if not f.startswith("-DTORCH_EXTENSION_NAME")]
        bf = ex.submit(_compile, "torch/bindings.cpp",
                       HOSTFLAGS + base + ["-Wno-unused-function", f"-DTORCH_EXTENSION_NAME=_C_{name}"], tag, False)
        objs = [f.result() for f in kf + hf + rf] + [bf.result()]
    out = PKG / f"_C_{name}{ext}"
    hiplink = [f"--offload-arch={ARCH}", "-fopenmp", f"-L{ROCM}/lib", "-lamdhip64"]
    _run([HIPCC, "-shared", "-o", str(out)] + [str(o) for o in objs] + hiplink + tld + ["-lrccl"])
    return out


def build_asan() -> Path:
    """Host-only sanitizer build of the CPU unit tests (kd-tree, brute force, CPU grid solver,
    .xyz I/O, checker): ``bin/knn_unit_asan`` with AddressSanitizer + UBSan (g++). GPU code is
    not sanitized (GPU ASan / XNACK are unavailable on the MI355X pool)."""
    san = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]
    flags = [f for f in HOSTFLAGS if f != "-O3"] + san + ["-DKN_UNIT_CPU_ONLY=1"]
    objs = [_compile(h, flags, "asan", False) for h in HOST]
    objs.append(_compile("tools/knn_unit.cpp", flags, "asan", False))
    exe = ROOT / "bin" / "knn_unit_asan"
    exe.parent.mkdir(exist_ok=True)
    _run([CXX, "-o", str(exe)] + [str(o) for o in objs] + san + ["-fopenmp"])
    return exe


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--asan", action="store_true", help="also build bin/knn_unit_asan (host ASan + UBSan)")
    a = ap.parse_args(argv)
    build(a.jobs, a.force)
    if a.asan:
        print(f"[build] asan: {build_asan()}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
