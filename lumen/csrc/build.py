"""Build lumen's native extension IN-TREE: ``lumen/_C<ext-suffix>.so``.

* every ``kernels/*.hip`` is compiled by ``hipcc --offload-arch=gfx950`` (CDNA4 only: no other
  targets, no CUDA, no hipify) -- these translation units include only HIP headers, so they
  rebuild in seconds;
* ``cpu/cpu_adam.cpp`` (host AdamW for ZeRO-Offload) by the host compiler with OpenMP;
* ``binding.cpp`` (pybind11 + torch headers, the slow one) only when it changed;
* linked into one shared object next to ``lumen/__init__.py`` so it travels with the repo
  snapshot to the GPU box (no JIT cache under ~/.cache).

Usage: ``python -m lumen.csrc.build [-j N] [--force] [--asm]``.
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys
import sysconfig
import time
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
BUILD = os.path.join(PKG, "..", "build", "lumen_native")
ARCH = os.environ.get("LUMEN_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "_C" + suffix)


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce

    inc = ce.include_paths()
    libdir = ce.library_paths()[0]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    import pybind11

    cflags = [f"-I{p}" for p in inc] + [f"-I{pybind11.get_include()}",
                                         f"-I{sysconfig.get_paths()['include']}",
                                         f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                                         "-DTORCH_EXTENSION_NAME=_C", "-DUSE_ROCM=1",
                                         "-D__HIP_PLATFORM_AMD__=1"]
    ldflags = [f"-L{libdir}", f"-Wl,-rpath,{libdir}", "-lc10", "-lc10_hip", "-ltorch",
               "-ltorch_cpu", "-ltorch_hip", "-ltorch_python"]
    return cflags, ldflags


def sources() -> list:
    """Every source the extension is built from (kernels, headers, host code, binding)."""
    return sorted(glob.glob(os.path.join(HERE, "kernels", "*.hip"))
                  + glob.glob(os.path.join(HERE, "kernels", "*.h"))
                  + [os.path.join(HERE, "cpu", "cpu_adam.cpp"), os.path.join(HERE, "binding.cpp")])


def source_digest() -> dict:
    """{relative path: sha256} of ``sources()`` and their combined digest."""
    import hashlib

    files = {}
    for f in sources():
        with open(f, "rb") as fh:
            files[os.path.relpath(f, PKG)] = hashlib.sha256(fh.read()).hexdigest()
    total = hashlib.sha256("".join(f"{k}:{v};" for k, v in sorted(files.items())).encode())
    return {"sha256": total.hexdigest(), "files": files}


def manifest_path(out: str = None) -> str:
    out = out or ext_path()
    return os.path.join(os.path.dirname(out), "_C.sources.json")


def read_manifest(out: str = None):
    import json

    try:
        with open(manifest_path(out)) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def _newer(src_list, obj):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(s) > t for s in src_list)


def _run(cmd):
    """Run a compile / link; its ``-o`` target is written under a temporary name and renamed
    on success, so an interrupted build never leaves a truncated object that looks current."""
    t0 = time.time()
    cmd = list(cmd)
    i = cmd.index("-o") + 1
    final = cmd[i]
    cmd[i] = tmp = f"{final}.part{os.getpid()}"
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        if os.path.exists(tmp):
            os.remove(tmp)
        raise RuntimeError(f"compile failed: {final}")
    os.replace(tmp, final)
    return time.time() - t0, r.stderr


def build(jobs: int = 8, force: bool = False, asm: bool = False, verbose: bool = True,
          build_dir: str = None, out: str = None) -> str:
    """Compile + link under an exclusive file lock next to the output ``.so``.

    Several processes may call this at once (every rank of a ``torch.distributed.run`` job whose
    extension is missing): the first one builds, the others block on the lock and then find
    everything up to date.  The link writes a temporary file that is renamed over the output,
    so no process can ever load a half-written shared object."""
    import fcntl

    build_dir = build_dir or os.environ.get("LUMEN_BUILD_DIR") or BUILD
    out = out or ext_path()
    os.makedirs(build_dir, exist_ok=True)
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out + ".lock", "a+") as lk:
        t0 = time.time()
        fcntl.flock(lk.fileno(), fcntl.LOCK_EX)
        if verbose and time.time() - t0 > 1.0:
            print(f"[lumen.build] waited {time.time() - t0:.1f}s for a concurrent build", flush=True)
        try:
            return _build_locked(jobs, force, asm, verbose, build_dir, out)
        finally:
            fcntl.flock(lk.fileno(), fcntl.LOCK_UN)


def _build_locked(jobs, force, asm, verbose, build_dir, out) -> str:
    headers = glob.glob(os.path.join(HERE, "kernels", "*.h"))
    common = ["-O3", "-fPIC", "-std=c++17"]
    jobs_list = []
    objs = []
    for src in sorted(glob.glob(os.path.join(HERE, "kernels", "*.hip"))):
        obj = os.path.join(build_dir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer([src] + headers, obj):
            cmd = [HIPCC, f"--offload-arch={ARCH}", "-munsafe-fp-atomics", *common, "-c", src,
                   "-o", obj]
            if asm:
                cmd.insert(1, "-save-temps")
            jobs_list.append(cmd)
    cpu_src = os.path.join(HERE, "cpu", "cpu_adam.cpp")
    cpu_obj = os.path.join(build_dir, "cpu_adam.o")
    objs.append(cpu_obj)
    if force or _newer([cpu_src], cpu_obj):
        jobs_list.append(["g++", "-O3", "-fPIC", "-std=c++17", "-fopenmp", "-c", cpu_src, "-o",
                          cpu_obj])
    bind_src = os.path.join(HERE, "binding.cpp")
    bind_obj = os.path.join(build_dir, "binding.o")
    objs.append(bind_obj)
    cflags, ldflags = _torch_flags()
    if force or _newer([bind_src], bind_obj):
        # host-only translation unit: plain g++ against the HIP host API headers
        jobs_list.append(["g++", "-O2", "-fPIC", "-std=c++17", f"-I{ROCM}/include", *cflags, "-c",
                          bind_src, "-o", bind_obj])
    if jobs_list:
        with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            for cmd, (dt, _) in zip(jobs_list, ex.map(_run, jobs_list)):
                if verbose:
                    print(f"[lumen.build] {os.path.basename(cmd[-3] if cmd[-2] == '-o' else cmd[-1])}"
                          f" {dt:.1f}s", flush=True)
    dig = source_digest()
    man = read_manifest(out)
    if (jobs_list or not os.path.exists(out) or _newer(objs, out) or man is None
            or man.get("sha256") != dig["sha256"]):
        # atomic rename inside _run: a concurrent loader sees the old or the new file
        _run([HIPCC, "-shared", "-fPIC", "-fopenmp", *objs, "-o", out, *ldflags])
        if verbose:
            print(f"[lumen.build] linked {out}", flush=True)
        # provenance: which sources this shared object was built from (checked at load time,
        # lumen.ops._native: a stale extension on a GPU box fails loudly)
        import json
        import platform

        tmp = manifest_path(out) + f".part{os.getpid()}"
        with open(tmp, "w") as f:
            json.dump(dict(dig, arch=ARCH, host=platform.node(),
                           built_at=time.strftime("%Y-%m-%dT%H:%M:%S"),
                           so_bytes=os.path.getsize(out)), f, indent=1)
        os.replace(tmp, manifest_path(out))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=int(os.environ.get("MAX_JOBS", "8")))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--asm", action="store_true", help="keep .s (-save-temps) for inspection")
    a = ap.parse_args()
    build(jobs=a.jobs, force=a.force, asm=a.asm)


if __name__ == "__main__":
    main()
