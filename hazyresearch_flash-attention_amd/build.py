"""Build libfa_hip.so in-tree for gfx950 with hipcc (no cmake, no torch extension machinery), and
the compiled fwd/bwd binding flash_attn/_fa_C.so over it (g++ against torch's headers).

    python hazyresearch_flash-attention_amd/build.py [--jobs N] [--force]

Each head-dim tile is its own translation unit so the template instantiations compile in
parallel. The shared object lands next to the Python package (flash_attn/libfa_hip.so), which
is where flash_attn/flash_attn_hip.py loads it from.
"""
import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
# A/B builds (tools only): FA_BUILD_DIR / FA_BUILD_OUT redirect the objects and the library,
# FA_EXTRA_CFLAGS adds compile flags (e.g. -DFA_BWD_XCD=0); the product build leaves them unset
BUILD = os.environ.get("FA_BUILD_DIR", os.path.join(HERE, "build"))
DEFAULT_OUT = os.path.join(HERE, "flash_attn", "libfa_hip.so")
OUT = os.environ.get("FA_BUILD_OUT", DEFAULT_OUT)
EXTRA_CFLAGS = os.environ.get("FA_EXTRA_CFLAGS", "").split()
# backward timing probes compute wrong gradients: they need an explicit probe build, and never
# into the product library's path
_PROBE_FLAGS = [f for f in EXTRA_CFLAGS if "PROBE" in f and not f.endswith("PROBE=0")]
if _PROBE_FLAGS and ("-DFA_AB_PROBE_BUILD" not in EXTRA_CFLAGS or OUT == DEFAULT_OUT):
    raise SystemExit(f"build.py: {' '.join(_PROBE_FLAGS)} is a timing probe (wrong results by design): "
                     "build it only with -DFA_AB_PROBE_BUILD and FA_BUILD_OUT set to a variant library")

KERNEL_TUS = ["fa_d32_fwd.hip", "fa_d64_fwd.hip", "fa_d128_fwd.hip", "fa_d32_bwd.hip", "fa_d64_bwd.hip", "fa_d128_bwd.hip"]
SOURCES = ["fa_api.cpp", "fa_asm.cpp", "fa_aux.hip", "fa_padding.hip", "fa_rotary.hip"] + KERNEL_TUS
# hand-scheduled assembly kernels: generator script -> .s -> code object -> embedded byte array
ASM_GEN = os.path.join(CSRC, "asm", "gen_fwd.py")
# (dtype, head-dim tile, waves per workgroup or "p" = the persistent 4-wave form, symbol)
ASM_KERNELS = [("bf16", 64, 4, "fa_asm_fwd_d64_bf16"), ("f16", 64, 4, "fa_asm_fwd_d64_f16"),
               ("bf16", 128, 4, "fa_asm_fwd_d128_bf16"), ("f16", 128, 4, "fa_asm_fwd_d128_f16"),
               ("bf16", 64, "p", "fa_asm_fwd_d64p_bf16"), ("f16", 64, "p", "fa_asm_fwd_d64p_f16"),
               ("bf16", 128, "p", "fa_asm_fwd_d128p_bf16"), ("f16", 128, "p", "fa_asm_fwd_d128p_f16"),
               ("bf16", 96, 4, "fa_asm_fwd_d96_bf16"), ("f16", 96, 4, "fa_asm_fwd_d96_f16"),
               ("bf16", 96, "p", "fa_asm_fwd_d96p_bf16"), ("f16", 96, "p", "fa_asm_fwd_d96p_f16"),
               ("bf16", 32, 4, "fa_asm_fwd_d32_bf16"), ("f16", 32, 4, "fa_asm_fwd_d32_f16"),
               ("bf16", 32, "p", "fa_asm_fwd_d32p_bf16"), ("f16", 32, "p", "fa_asm_fwd_d32p_f16")]
LLVM_BIN = "/opt/rocm/lib/llvm/bin"
# Per-source machine-scheduler choice, from one-process A/Bs of every LLVM AMDGPU strategy
# (DESIGN 7.4): the forward kernels with the AMDGPU register-pressure trackers (north star +2 %,
# C2 +4 %), the D=32 and D=128 backward with the iterative ILP scheduler (-5 %, -2…3 %); the D=64
# backward keeps the default (every alternative even or slower on C3).
_TRACKERS = ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"]
_ITILP = ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]
SOURCE_FLAGS = {
    "fa_d32_fwd.hip": _TRACKERS, "fa_d64_fwd.hip": _TRACKERS, "fa_d128_fwd.hip": _TRACKERS,
    "fa_d32_bwd.hip": _ITILP, "fa_d128_bwd.hip": _ITILP,
}
ARCH = os.environ.get("FA_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def common_flags():
    return ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", INCLUDE, "-I", CSRC,
            "-mllvm", "-amdgpu-mfma-vgpr-form",  # keep MFMA C/D in VGPRs: no accvgpr shuffles
            "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]


def _newer(target, deps):
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def _deps():
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hdrs.append(os.path.join(INCLUDE, "fa_hip.h"))
    return hdrs + [os.path.abspath(__file__)]


def compile_one(src, force=False, extra=()):
    os.makedirs(BUILD, exist_ok=True)
    obj = os.path.join(BUILD, src + ".o")
    srcp = os.path.join(CSRC, src)
    if not force and _newer(obj, [srcp] + _deps()):
        return obj
    lang = ["-x", "hip"] if src.endswith(".hip") else ["-x", "hip"]
    cmd = [hipcc()] + common_flags() + SOURCE_FLAGS.get(src, []) + EXTRA_CFLAGS + list(extra) + lang + ["-c", srcp, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build_asm(force=False):
    """Generate, assemble and link each assembly kernel, then embed the code objects in one C++
    source (byte arrays) that is compiled into the library."""
    os.makedirs(BUILD, exist_ok=True)
    blob_cpp = os.path.join(BUILD, "fa_asm_blobs.cpp")
    if not force and _newer(blob_cpp, [ASM_GEN, os.path.abspath(__file__)]):
        return blob_cpp
    parts = ["// generated by build.py from csrc/asm/gen_fwd.py: gfx950 code objects\n"]
    for dt, hd, nw, sym in ASM_KERNELS:
        asm = os.path.join(BUILD, sym + ".s")
        obj = os.path.join(BUILD, sym + ".o")
        hsaco = os.path.join(BUILD, sym + ".hsaco")
        form = ["--persist", "1"] if nw == "p" else ["--waves", str(nw)]
        # FA_ASM_GEN_FLAGS: extra generator switches for a variant library (A/B tools only)
        extra = os.environ.get("FA_ASM_GEN_FLAGS", "").split()
        extra += os.environ.get(f"FA_ASM_GEN_FLAGS_D{hd}", "").split()     # one tile only
        _run([sys.executable, ASM_GEN, "--dtype", dt, "--hd", str(hd)] + form + extra + ["--out", asm])
        _run([os.path.join(LLVM_BIN, "clang"), "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
              f"-mcpu={ARCH}", "-c", asm, "-o", obj])
        _run([os.path.join(LLVM_BIN, "ld.lld"), "-shared", obj, "-o", hsaco])
        data = open(hsaco, "rb").read()
        body = ",".join(str(b) for b in data)
        parts.append(f'extern "C" const unsigned char {sym}[] __attribute__((aligned(4096))) = {{{body}}};\n')
        parts.append(f'extern "C" const unsigned long {sym}_size = {len(data)}ul;\n')
    with open(blob_cpp, "w") as f:
        f.write("".join(parts))
    return blob_cpp


def compile_blob(blob_cpp, force=False):
    obj = blob_cpp + ".o"
    if not force and _newer(obj, [blob_cpp]):
        return obj
    _run([hipcc(), "-O1", "-fPIC", "-c", "-x", "c++", blob_cpp, "-o", obj])
    return obj


TORCH_EXT_SRC = os.path.join(CSRC, "fa_torch.cpp")
TORCH_EXT_OUT = os.path.join(HERE, "flash_attn", "_fa_C.so")


def build_torch_ext(force=False):
    """The compiled fwd/bwd binding (csrc/fa_torch.cpp): a host-only pybind11 module over the C ABI,
    linked against the in-tree libfa_hip.so (rpath $ORIGIN) and torch's libraries."""
    deps = [TORCH_EXT_SRC, os.path.join(INCLUDE, "fa_hip.h"), OUT, os.path.abspath(__file__)]
    if not force and _newer(TORCH_EXT_OUT, deps):
        return TORCH_EXT_OUT
    import sysconfig
    import torch
    tdir = os.path.dirname(torch.__file__)
    abi = int(getattr(torch._C, "_GLIBCXX_USE_CXX11_ABI", True))
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-fPIC", "-shared",
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_fa_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
           "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM",
           "-I", os.path.join(tdir, "include"), "-I", os.path.join(tdir, "include", "torch", "csrc", "api", "include"),
           "-I", sysconfig.get_paths()["include"], "-I", "/opt/rocm/include", "-I", INCLUDE,
           TORCH_EXT_SRC, "-o", TORCH_EXT_OUT,
           "-L", os.path.join(tdir, "lib"), "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_python",
           "-L", os.path.dirname(OUT), "-l:libfa_hip.so", "-Wl,-rpath,$ORIGIN"]
    _run(cmd)
    return TORCH_EXT_OUT


def build(jobs=None, force=False, verbose=True):
    jobs = jobs or min(len(SOURCES), os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        fut_asm = ex.submit(lambda: compile_blob(build_asm(force), force))
        objs = list(ex.map(lambda s: compile_one(s, force), SOURCES))
        objs.append(fut_asm.result())
    if force or not _newer(OUT, objs):
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"built {OUT}")
    if OUT == DEFAULT_OUT:
        build_torch_ext(force)
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    args = ap.parse_args()
    try:
        build(args.jobs, args.force)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
