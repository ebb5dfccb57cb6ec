"""In-tree build of the HIP extension (``pytorch_dppo_amd/ops/_dppo_hip*.so``).

No JIT cache, no hipify, no setuptools: each ``csrc/*.hip`` is compiled by ``hipcc
--offload-arch=gfx950`` to an object (cached by content hash under ``build/``), the torch
binding ``csrc/bindings.cpp`` is compiled once with the torch include paths, and everything
is linked into one shared object next to this file, so it travels to the GPU box with the
repo snapshot and is what ``import`` loads there.

    python -m pytorch_dppo_amd.ops._build        # or: __graft_entry__.build()
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build")
OUT_DIR = os.path.dirname(os.path.abspath(__file__))
EXT_NAME = "_dppo_hip"
ARCH = os.environ.get("DPPO_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
DEVICE_SRCS = ["rollout.hip", "mlp.hip", "mlp_head.hip", "phead.hip", "wgrad.hip", "optim.hip", "obs.hip"]
HOST_SRCS = ["bindings.cpp", "comm.cpp"]   # compiled with the torch include paths
HEADERS = ["common.h", "mlp_core.h", "kernels.h", "t32.h"]


def ext_path(variant: str = "") -> str:
    name = EXT_NAME + (f"_{variant}" if variant else "")
    return os.path.join(OUT_DIR, name + sysconfig.get_config_var("EXT_SUFFIX"))


def _torch_flags(ext_name: str = EXT_NAME):
    import torch
    from torch.utils import cpp_extension as ce
    inc = ce.include_paths(device_type="cuda")
    libdirs = ce.library_paths(device_type="cuda")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cflags = [f"-I{p}" for p in inc] + [f"-I{sysconfig.get_paths()['include']}",
                                         f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                                         f"-DTORCH_EXTENSION_NAME={ext_name}",
                                         "-DTORCH_API_INCLUDE_EXTENSION_H", "-DUSE_ROCM=1"]
    ldflags = [f"-L{p}" for p in libdirs] + [f"-Wl,-rpath,{p}" for p in libdirs] + [
        "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip",
        "-lrccl"]   # torch's own librccl.so (first -L): one RCCL in the process (csrc/comm.cpp)
    return cflags, ldflags


def _digest(paths, extra: str) -> str:
    h = hashlib.sha256(extra.encode())
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _compile(src: str, cflags, verbose: bool, csrc: str = CSRC, extra=()) -> str:
    srcp = os.path.join(csrc, src)
    deps = [srcp] + [os.path.join(csrc, h) for h in HEADERS]
    # -amdgpu-mfma-vgpr-form: MFMA accumulators in ordinary VGPRs (gfx90a+ unified register
    # file).  With AGPR accumulators the allocator shuffled them through VGPRs every loop turn
    # (~1,600 v_accvgpr_* in mlp_train, 96 per wgrad k-step pair); with it those copies vanish.
    base = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result",
            "-mllvm", "-amdgpu-mfma-vgpr-form"]
    # A/B builds of compile-time variants (e.g. DPPO_EXTRA_CFLAGS="-DDPPO_X_CACHED"); the
    # flags enter the object cache key, so switching back rebuilds nothing stale
    base += os.environ.get("DPPO_EXTRA_CFLAGS", "").split() + list(extra)
    flags = base + cflags
    key = _digest(deps, " ".join(flags))
    obj = os.path.join(BUILD, f"{os.path.splitext(src)[0]}-{key}.o")
    if os.path.exists(obj):
        return obj
    cmd = [HIPCC] + flags + ["-c", srcp, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    return obj


def build(verbose: bool = False, force: bool = False, variant: str = "", csrc: str = CSRC, defines=()) -> str:
    """Build the extension.  ``variant`` + ``csrc`` / ``defines`` (A/B diagnostics): the same
    bindings built from another source tree (e.g. an earlier commit's csrc/) or with extra -D
    macros as module ``_dppo_hip_<variant>``, loadable next to the default one (ops/native.py
    load_variant) so kernel versions can be timed interleaved in one process on one box."""
    os.makedirs(BUILD, exist_ok=True)
    tcflags, ldflags = _torch_flags(EXT_NAME + (f"_{variant}" if variant else ""))
    jobs = [(s, []) for s in DEVICE_SRCS] + [(s, tcflags) for s in HOST_SRCS]
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        extra = [f"-D{d}" for d in defines]
        objs = list(ex.map(lambda j: _compile(j[0], j[1], verbose, csrc, extra), jobs))
    out = ext_path(variant)
    # the object names carry their source digests (hipcc's object bytes are not reproducible
    # across machines), so the stamp names the sources + flags the .so was built from
    key = hashlib.sha256((" ".join(os.path.basename(o) for o in objs) + " "
                          + " ".join(ldflags)).encode()).hexdigest()[:16]
    stamp = out + ".stamp"
    if not force and os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == key:
        return out
    tmp = out + ".tmp.so"
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}"] + objs + ldflags + ["-o", tmp]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(key)
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    var = args[args.index("--variant") + 1] if "--variant" in args else ""
    src = args[args.index("--src") + 1] if "--src" in args else CSRC
    defs = args[args.index("--define") + 1].split(",") if "--define" in args else []
    p = build(verbose="-v" in args, force="--force" in args, variant=var, csrc=src, defines=defs)
    print(p)
