"""In-tree build of the native extension ``gaussiank_sgd_amd/_C.so``.

No hipify, no JIT cache: HIP kernels are compiled with ``hipcc
--offload-arch=gfx950`` and the torch-op bindings / RCCL engine with g++ against
the torch headers, then linked into one shared object next to the package so
it travels to the GPU box with the source tree.

Objects are cached under ``build/`` keyed by a hash of (source, headers,
flags); ``python -m gaussiank_sgd_amd.ops.build`` rebuilds what changed.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path
from typing import List

PKG = Path(__file__).resolve().parents[1]
REPO = PKG.parent
CSRC = PKG / "ops" / "csrc"
BUILD = REPO / "build" / "gksgd_ext"
TARGET = PKG / "_C.so"
# host-sanitizer variant (python -m gaussiank_sgd_amd.ops.build --asan): the C++
# bindings / RCCL engine and the host side of every .hip file are built with
# AddressSanitizer + UBSan; device code is unchanged (GPU ASan is not used)
ASAN = os.environ.get("GKSGD_ASAN", "0") == "1"
if ASAN:
    BUILD = REPO / "build" / "gksgd_ext_asan"
    TARGET = REPO / "build" / "asan" / "_C.so"
SAN_HOST = ["-fsanitize=address", "-fsanitize=undefined"]
# A/B variants: GKSGD_VARIANT=<name> builds variants/<name>/_C.so with the extra
# hipcc flags of GKSGD_VARIANT_FLAGS (e.g. "-DGK_BN_UNROLL=1"); load it with
# GKSGD_EXT=variants/<name>/_C.so (under variants/: build/ is not sent to the GPU box)
VARIANT = os.environ.get("GKSGD_VARIANT", "")
VARIANT_FLAGS = os.environ.get("GKSGD_VARIANT_FLAGS", "").split()
if VARIANT and not ASAN:
    BUILD = REPO / "build" / ("gksgd_ext_" + VARIANT)
    TARGET = REPO / "variants" / VARIANT / "_C.so"
ARCH = os.environ.get("GKSGD_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

HIP_SOURCES = [
    "kernels/compress.hip",
    "kernels/scatter.hip",
    "kernels/optim.hip",
    "kernels/bn_act.hip",
    "kernels/gemm.hip",
    # gemm_inst.hip: one object per GEMM instantiation unit (-DGK_GEMM_UNIT=<n>, gemm_kern.h)
    *["kernels/gemm_inst.hip#%d" % u for u in range(11)],
    "kernels/ln.hip",
    "kernels/linear.hip",
    "kernels/lstm.hip",
    "kernels/stem.hip",
    "kernels/wgrad3.hip",
    "kernels/attn.hip",
    "kernels/attn_f32.hip",
    "kernels/embed.hip",
    "kernels/xent.hip",
    "kernels/winograd.hip",
    "kernels/wino_x6.hip",
    "kernels/stem_f32.hip",
    "kernels/prep.hip",
]
CXX_SOURCES = [
    "comm/rccl_engine.cpp",
    "bindings.cpp",
]
HEADERS = ["kernels/common.h", "kernels/gk_kernels.h", "kernels/mfma_util.h", "kernels/gemm_kern.h",
           "kernels/wino_x6_common.h",
           "comm/rccl_engine.h"]
# per-file extra flags: the sparse aggregation must round product and sum
# separately (bit-identical to the reference arithmetic and the CPU mirror)
# the GEMM units: no SLP vectorisation -- packed fp32 VALU (v_pk_add_f32) beside
# MFMAs costs more issue cycles than scalar pairs (MI355X_MICROARCH.md constants);
# measured on the bf16x6 split: GEMMs 2.5-4.5% faster (r5c20)
EXTRA_FLAGS = {"kernels/scatter.hip": ["-ffp-contract=off"], "kernels/gemm_inst.hip": ["-fno-slp-vectorize"]}


def _torch_dirs():
    import torch  # noqa: F401  (only for paths)
    tdir = Path(torch.__file__).resolve().parent
    return tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include", tdir / "lib"


def _hipcc() -> str:
    p = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    return p


def _hip_flags() -> List[str]:
    san = []
    if ASAN:
        for f in SAN_HOST:
            san += ["-Xarch_host", f]
        san += ["-Xarch_host", "-fno-omit-frame-pointer"]
    return san + VARIANT_FLAGS + [
        "--offload-arch=" + ARCH,
        "-O3",
        "-fPIC",
        "-std=c++17",
        "-munsafe-fp-atomics",
        "-Wno-unused-result",
        "-I" + str(CSRC),
        "-I" + str(CSRC / "kernels"),
    ]


def _cxx_flags() -> List[str]:
    inc, api_inc, _ = _torch_dirs()
    import torch
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return (SAN_HOST + ["-fno-omit-frame-pointer", "-g"] if ASAN else []) + [
        "-O2",
        "-fPIC",
        "-std=c++17",
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        "-D_GLIBCXX_USE_CXX11_ABI=%d" % abi,
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-Wno-deprecated-declarations",
        "-Wno-unused-parameter",
        "-I" + str(CSRC),
        "-I" + str(inc),
        "-I" + str(api_inc),
        "-I" + os.path.join(ROCM, "include"),
        "-I" + sysconfig.get_paths()["include"],
    ]


def _digest(src: Path, flags: List[str]) -> str:
    h = hashlib.sha256()
    h.update(src.read_bytes())
    for hd in HEADERS:
        p = CSRC / hd
        if p.exists():
            h.update(p.read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _compile(src_rel: str, kind: str, verbose: bool) -> Path:
    # "<file>#<n>": instantiation unit n of a file compiled once per unit (-DGK_GEMM_UNIT=n)
    src_rel, _, unit = src_rel.partition("#")
    src = CSRC / src_rel
    if kind == "hip":
        cc, flags = _hipcc(), _hip_flags()
    else:
        cc, flags = os.environ.get("CXX", "g++"), _cxx_flags()
    flags = flags + EXTRA_FLAGS.get(src_rel, []) + (["-DGK_GEMM_UNIT=" + unit] if unit else [])
    tag = src_rel.replace("/", "_") + ("." + unit if unit else "")
    obj = BUILD / (tag + "." + _digest(src, flags) + ".o")
    if obj.exists():
        return obj
    BUILD.mkdir(parents=True, exist_ok=True)
    cmd = [cc] + flags + ["-c", str(src), "-o", str(obj) + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("compile failed for %s:\n%s\n%s" % (src_rel, r.stdout, r.stderr))
    os.replace(str(obj) + ".tmp", obj)
    return obj


def build(verbose: bool = False, force: bool = False, jobs: int = 0) -> Path:
    # the GEMM units dominate (minutes each): one job per CPU, at most 8
    jobs = jobs or min(8, os.cpu_count() or 4)
    if force and BUILD.exists():
        shutil.rmtree(BUILD)
    _, _, tlib = _torch_dirs()
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = [ex.submit(_compile, s, "hip", verbose) for s in HIP_SOURCES]
        futs += [ex.submit(_compile, s, "cxx", verbose) for s in CXX_SOURCES]
        objs = [f.result() for f in futs]
    link_key = hashlib.sha256("|".join(str(o) for o in objs).encode()).hexdigest()[:16]
    stamp = BUILD / ("link." + link_key)
    if TARGET.exists() and stamp.exists() and not force:
        return TARGET
    TARGET.parent.mkdir(parents=True, exist_ok=True)
    cmd = [os.environ.get("CXX", "g++"), "-shared", "-o", str(TARGET) + ".tmp"] + (SAN_HOST if ASAN else []) + \
        [str(o) for o in objs] + [
        "-L" + str(tlib),
        "-Wl,-rpath," + str(tlib),
        "-L" + os.path.join(ROCM, "lib"),
        "-ltorch",
        "-ltorch_cpu",
        "-lc10",
        "-lc10_hip",
        "-ltorch_hip",
        "-lamdhip64",
        "-lrccl",
    ]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n%s\n%s" % (r.stdout, r.stderr))
    os.replace(str(TARGET) + ".tmp", TARGET)
    for old in BUILD.glob("link.*"):
        old.unlink()
    stamp.write_text("ok")
    return TARGET


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    ap.add_argument("--asan", action="store_true", help="host ASan+UBSan variant under build/asan/ (re-execs)")
    args = ap.parse_args(argv)
    if args.asan and not ASAN:
        env = dict(os.environ, GKSGD_ASAN="1")
        return subprocess.call([sys.executable, "-m", "gaussiank_sgd_amd.ops.build"] +
                               [a for a in (argv if argv is not None else sys.argv[1:]) if a != "--asan"], env=env)
    out = build(verbose=args.verbose, force=args.force, jobs=args.jobs)
    print(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
