"""In-tree native build for k8s_amd.

Builds two native artefacts, both in-tree so they travel with the repo
snapshot to the GPU box:

* ``k8s_amd/_C*.so``      -- gfx950 HIP kernels + PyTorch bindings. Each
  ``csrc/kernels/*.hip`` file is compiled by ``hipcc --offload-arch=gfx950``
  WITHOUT torch headers (seconds per file, in parallel); only
  ``csrc/ops_binding.cpp`` sees the torch headers. Linked against torch's own
  ``libamdhip64`` so the extension shares PyTorch's HIP runtime and streams.
* ``k8s_amd/_operator*.so`` + ``bin/tf_operator`` + ``bin/e2e`` -- the C++17
  control plane (see csrc/operator), built with g++.

Usage: ``python -m k8s_amd._build [--force] [--only kernels|operator]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(ROOT)
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(REPO, "build")
ARCH = os.environ.get("K8S_AMD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _torch_dirs():
    import torch  # noqa: deferred, heavy

    tdir = os.path.dirname(torch.__file__)
    return (
        [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")],
        os.path.join(tdir, "lib"),
    )


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed (%d): %s\n%s" % (r.returncode, " ".join(cmd), r.stdout))
    return r.stdout


HIP_FLAGS = [
    "--offload-arch=" + ARCH,
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-munsafe-fp-atomics",
    "-Wno-unused-result",
    # every `#pragma unroll` over register-resident tiles (MFMA accumulators, epilogue statistics) must
    # unroll fully: past LLVM's default pragma threshold a big epilogue silently stays rolled and the
    # dynamically indexed accumulator array moves to scratch memory (a 3x slowdown seen on gfx950)
    "-mllvm",
    "-pragma-unroll-threshold=1000000",
]

# Kernels must not use scratch (private) memory: checked on every kernel build from the compiler's
# resource-usage remarks, written to build/kernel_resources.txt.
RESOURCE_FLAG = "-Rpass-analysis=kernel-resource-usage"


def parse_resource_usage(text: str) -> dict:
    """{kernel symbol: {"VGPRs": n, "AGPRs": n, "ScratchSize": n, "Occupancy": n, ...}} from hipcc remarks."""
    out, cur = {}, None
    for line in text.splitlines():
        if "remark:" not in line:
            continue
        body = line.split("remark:", 1)[1].split("[-Rpass", 1)[0].strip()
        if body.startswith("Function Name:"):
            cur = out.setdefault(body.split(":", 1)[1].strip(), {})
        elif cur is not None and ":" in body:
            k, v = body.split(":", 1)
            k = k.split("[")[0].strip()
            try:
                cur[k] = int(v.strip())
            except ValueError:
                cur[k] = v.strip()
    return out


def kernel_sources():
    return sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))


def build_kernels(force=False, jobs=None) -> str:
    inc, tlib = _torch_dirs()
    os.makedirs(os.path.join(BUILD, "obj"), exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    objs, jobs_list = [], []
    for src in kernel_sources():
        obj = os.path.join(BUILD, "obj", os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + headers):
            jobs_list.append([HIPCC, *HIP_FLAGS, RESOURCE_FLAG, "-I", os.path.join(CSRC, "kernels"), "-c", src,
                              "-o", obj])
    bind_src = os.path.join(CSRC, "ops_binding.cpp")
    bind_obj = os.path.join(BUILD, "obj", "ops_binding.o")
    objs.append(bind_obj)
    if force or _newer(bind_obj, [bind_src] + headers):
        flags = [
            "-DUSE_ROCM=1",
            "-D__HIP_PLATFORM_AMD__=1",
            "-DTORCH_EXTENSION_NAME=_C",
            "-DTORCH_API_INCLUDE_EXTENSION_H",
            "-D_GLIBCXX_USE_CXX11_ABI=1",
            "-Wno-deprecated-declarations",
        ]
        incs = sum([["-I", d] for d in inc + [sysconfig.get_paths()["include"], CSRC]], [])
        jobs_list.append([HIPCC, *HIP_FLAGS, *flags, *incs, "-c", bind_src, "-o", bind_obj])
    n = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=n) as ex:
        logs = [(j, fut.result()) for j, fut in [(j, ex.submit(_run, j)) for j in jobs_list]]
    try:
        _check_resources(logs)
    except RuntimeError:
        for j in jobs_list:  # a spilling object must not survive to be linked by the next (incremental) build
            o = j[j.index("-o") + 1]
            if os.path.exists(o):
                os.remove(o)
        raise
    out = os.path.join(ROOT, "_C" + _ext_suffix())
    if force or jobs_list or not os.path.exists(out) or _newer(out, objs):
        libs = ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lamdhip64"]
        tmp = out + ".tmp"
        _run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", *objs, "-o", tmp, "-L", tlib, *libs,
              "-Wl,-rpath," + tlib])
        os.replace(tmp, out)
    return out


def _check_resources(logs):
    """Record per-kernel resource usage; refuse kernels that spill to scratch."""
    report = os.path.join(BUILD, "kernel_resources.txt")
    usage = {}
    if os.path.exists(report):
        for line in open(report):
            parts = line.rstrip("\n").split("\t")
            if len(parts) == 2:
                usage[parts[0]] = parts[1]
    bad = []
    for cmd, text in logs:
        if RESOURCE_FLAG not in cmd:
            continue
        for name, r in parse_resource_usage(text).items():
            usage[name] = " ".join("%s=%s" % (k.replace(" ", ""), v) for k, v in sorted(r.items()))
            if r.get("ScratchSize", 0):
                bad.append("%s: %d B/lane scratch" % (name, r["ScratchSize"]))
    with open(report, "w") as f:
        for k in sorted(usage):
            f.write("%s\t%s\n" % (k, usage[k]))
    if bad and os.environ.get("K8S_AMD_ALLOW_SCRATCH") != "1":
        raise RuntimeError("kernels spill to scratch memory (see %s):\n  %s" % (report, "\n  ".join(bad)))


SANITIZERS = {"asan": "address,undefined", "tsan": "thread"}


def build_operator(force=False, sanitize=None) -> list:
    """Build the C++17 control plane (core library, pybind module, binaries).

    ``sanitize`` = "asan" (AddressSanitizer + UBSan) or "tsan" (ThreadSanitizer) builds the host-side
    binaries only, as ``bin/tf_operator-<san>`` / ``bin/e2e-<san>`` (separate object dir, -O1 -g,
    frame pointers, UBSan set to abort on the first report) for the sanitizer tests."""
    opdir = os.path.join(CSRC, "operator")
    if not os.path.isdir(opdir):
        return []
    srcs = sorted(glob.glob(os.path.join(opdir, "*.cc")))
    core = [s for s in srcs if not os.path.basename(s).startswith(("main_", "py_"))]
    hdrs = glob.glob(os.path.join(opdir, "*.h"))
    objdir = os.path.join(BUILD, "opobj" + ("-" + sanitize if sanitize else ""))
    os.makedirs(objdir, exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    base = ["-std=c++17", "-O2", "-fPIC", "-Wall", "-Wno-unused-function", "-I", opdir]
    extra = os.environ.get("K8S_AMD_OP_CFLAGS", "").split()
    if sanitize:
        base[1] = "-O1"
        extra += ["-g", "-fno-omit-frame-pointer", "-fsanitize=" + SANITIZERS[sanitize]]
        if sanitize == "asan":
            extra += ["-fno-sanitize-recover=undefined"]
        srcs = [x for x in srcs if not os.path.basename(x).startswith("py_")]
    jobs_list, objs = [], {}
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs[s] = o
        flags = list(base) + extra
        if os.path.basename(s).startswith("py_"):
            import pybind11

            flags += ["-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"], "-fvisibility=hidden"]
        if force or _newer(o, [s] + hdrs):
            jobs_list.append([cxx, *flags, "-c", s, "-o", o])
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        for fut in [ex.submit(_run, j) for j in jobs_list]:
            fut.result()
    outs = []
    core_objs = [objs[s] for s in core]
    libflags = ["-lssl", "-lcrypto", "-lpthread"] + extra
    for s in srcs:
        b = os.path.basename(s)
        if b.startswith("py_"):
            out = os.path.join(ROOT, "_operator" + _ext_suffix())
            _run([cxx, "-shared", "-fPIC", objs[s], *core_objs, "-o", out, *libflags])
            outs.append(out)
        elif b.startswith("main_"):
            os.makedirs(os.path.join(REPO, "bin"), exist_ok=True)
            out = os.path.join(REPO, "bin", b[len("main_"):-3] + ("-" + sanitize if sanitize else ""))
            _run([cxx, objs[s], *core_objs, "-o", out, *libflags])
            outs.append(out)
    return outs


def build_all(force=False, only=None):
    outs = []
    if only in (None, "operator"):
        outs += build_operator(force)
    if only in ("sanitizers",):
        for san in SANITIZERS:
            outs += build_operator(force, sanitize=san)
    if only in (None, "kernels"):
        outs.append(build_kernels(force))
    return outs


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["kernels", "operator", "sanitizers"])
    ap.add_argument("--clean", action="store_true")
    a = ap.parse_args(argv)
    if a.clean:
        shutil.rmtree(BUILD, ignore_errors=True)
    for o in build_all(a.force, a.only):
        print(o)


if __name__ == "__main__":
    sys.exit(main())
