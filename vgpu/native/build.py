"""Build every native artefact of the framework in-tree (no JIT cache).

Outputs go to ``vgpu/_lib/`` so they travel with the repository snapshot to a
GPU box.  Everything here cross-compiles on a CPU-only machine:

* ``libvgpu.so``          — in-container enforcement library (C++, LD_PRELOAD);
                            never links HIP (PyTorch ships its own runtime).
* ``libvgpu_smi.so``      — device discovery facade over amdsmi/sysfs (C++).
* ``libvgpu_kernels.so``  — hand-written gfx950 HIP kernels (hipcc).
* ``fakes/libamdhip64.so.7``, ``fakes/libhsa-runtime64.so.1``,
  ``fakes/libamd_smi.so`` — fixture-driven fake vendor runtimes for CPU tests.
* ``shim_driver``          — scenario driver linked against the fakes.

Usage: ``python -m vgpu.native.build [--sanitize thread|address] [targets...]``.
"""
from __future__ import annotations

import argparse
import hashlib
import os
import re
import shutil
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
NATIVE = REPO / "native"
OUT = REPO / "vgpu" / "_lib"
FAKES_OUT = OUT / "fakes"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("VGPU_OFFLOAD_ARCH", "gfx950")

CXX = os.environ.get("CXX", "g++")
HIPCC = str(ROCM / "bin" / "hipcc")

COMMON = ["-std=c++17", "-O2", "-fPIC", "-Wall", "-Wno-unused-parameter",
          "-D__HIP_PLATFORM_AMD__", f"-I{ROCM / 'include'}", f"-I{NATIVE / 'include'}"]

SHIM_SOURCES = sorted((NATIVE / "shim").glob("*.cpp"))


def _run(cmd: list[str], cwd: Path | None = None) -> None:
    print("+", " ".join(str(c) for c in cmd), flush=True)
    subprocess.run([str(c) for c in cmd], cwd=cwd, check=True)


def _stamp(target: Path, inputs: list[Path], extra: str = "") -> bool:
    """True when `target` is up to date w.r.t. `inputs` (content hash)."""
    h = hashlib.sha256(extra.encode())
    for p in inputs:
        h.update(p.read_bytes())
    digest = h.hexdigest()
    stamp = target.with_name(target.name + ".stamp")
    if target.exists() and stamp.exists() and stamp.read_text() == digest:
        return True
    stamp.parent.mkdir(parents=True, exist_ok=True)
    stamp.write_text("")  # invalidate until the build succeeds
    return False


def _mark(target: Path, inputs: list[Path], extra: str = "") -> None:
    h = hashlib.sha256(extra.encode())
    for p in inputs:
        h.update(p.read_bytes())
    target.with_name(target.name + ".stamp").write_text(h.hexdigest())


def _headers() -> list[Path]:
    return sorted((NATIVE / "include").rglob("*.h")) + sorted((NATIVE / "shim").glob("*.h"))


def build_shim(sanitize: str | None = None, force: bool = False) -> Path:
    OUT.mkdir(parents=True, exist_ok=True)
    name = "libvgpu.so" if not sanitize else f"libvgpu_{sanitize}.so"
    target = OUT / name
    inputs = SHIM_SOURCES + _headers()
    if not force and _stamp(target, inputs, str(sanitize)):
        return target
    flags = list(COMMON) + ["-fvisibility=hidden"]
    if sanitize:
        flags += [f"-fsanitize={sanitize}", "-g", "-O1"]
    link = ["-shared", "-ldl", "-lpthread"]
    if not sanitize:
        link.append("-Wl,--no-undefined")  # proves we never link the HIP runtime
    _run([CXX, *flags, *SHIM_SOURCES, "-o", target, *link])
    _mark(target, inputs, str(sanitize))
    return target


def build_smi(force: bool = False) -> Path:
    OUT.mkdir(parents=True, exist_ok=True)
    target = OUT / "libvgpu_smi.so"
    srcs = sorted((NATIVE / "smi").glob("*.cpp"))
    inputs = srcs + sorted((NATIVE / "smi").glob("*.h")) + _headers()
    if not force and _stamp(target, inputs):
        return target
    _run([CXX, *COMMON, "-fvisibility=hidden", *srcs, "-o", target, "-shared", "-ldl",
          "-lpthread", "-Wl,--no-undefined"])
    _mark(target, inputs)
    return target


def build_sched(force: bool = False) -> Path:
    """libvgpu_sched.so: the scheduler extender's native scoring core."""
    OUT.mkdir(parents=True, exist_ok=True)
    target = OUT / "libvgpu_sched.so"
    srcs = sorted((NATIVE / "sched").glob("*.cpp"))
    if not force and _stamp(target, srcs):
        return target
    _run([CXX, "-std=c++17", "-O3", "-fPIC", "-Wall", "-fvisibility=hidden", *srcs, "-o", target, "-shared",
          "-Wl,--no-undefined"])
    _mark(target, srcs)
    return target


def build_kernels(force: bool = False) -> Path:
    """hipcc --offload-arch=gfx950 → libvgpu_kernels.so (links libamdhip64.so.7,
    which resolves to the already-loaded PyTorch runtime in a torch process)."""
    OUT.mkdir(parents=True, exist_ok=True)
    target = OUT / "libvgpu_kernels.so"
    srcs = sorted((NATIVE / "kernels").glob("*.hip"))
    inputs = srcs + sorted((NATIVE / "kernels").glob("*.h"))
    if not force and _stamp(target, inputs, ARCH):
        return target
    _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
          "-fvisibility=hidden", f"-I{NATIVE / 'include'}", "-mcode-object-version=5",
          *srcs, "-o", target])
    _check_stubs(target)
    _mark(target, inputs, ARCH)
    return target


def _check_stubs(lib: Path) -> None:
    """A kernel template whose host-side instantiation fails substitution (e.g.
    a lambda capturing a local array of value-dependent size) links anyway,
    with an undefined launch stub, and only fails at dlopen on the GPU box.
    Refuse such a library here."""
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    out = subprocess.run([nm, "-D", "--undefined-only", str(lib)], capture_output=True, text=True).stdout
    bad = [ln.split()[-1] for ln in out.splitlines() if "__device_stub__" in ln]
    if bad:
        lib.unlink(missing_ok=True)
        raise RuntimeError(f"{lib.name}: undefined kernel launch stubs {bad}")


def build_probe_module(force: bool = False) -> Path:
    """hipcc --genco: a raw gfx950 code object (not a shared library) for the
    module-charging probe (hipModuleLoadData)."""
    OUT.mkdir(parents=True, exist_ok=True)
    target = OUT / "module_probe.hsaco"
    src = NATIVE / "probes" / "module_probe.hip"
    if not force and _stamp(target, [src], ARCH):
        return target
    _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "--genco", src, "-o", target])
    _mark(target, [src], ARCH)
    return target


def _hip_versions() -> dict[str, str]:
    """symbol -> version node of the real libamdhip64 (for the fake's version script)."""
    out: dict[str, str] = {}
    for lib in (ROCM / "lib" / "libamdhip64.so",):
        if not lib.exists():
            continue
        txt = subprocess.run(["nm", "-D", "--defined-only", str(lib)], capture_output=True,
                             text=True).stdout
        for line in txt.splitlines():
            m = re.match(r"\S+\s+T\s+(\w+)@@(\S+)", line)
            if m:
                out[m.group(1)] = m.group(2)
    return out


def _version_script(src: Path, default_node: str, versions: dict[str, str], extra_global: str) -> str:
    text = src.read_text()
    funcs = sorted(set(f for f in re.findall(r"^(?:hipError_t|hsa_status_t)\s+(\w+)\s*\(", text, re.M)
                       if f.startswith(("hip", "hsa"))))
    nodes: dict[str, list[str]] = {}
    for f in funcs:
        nodes.setdefault(versions.get(f, default_node), []).append(f)

    def key(v: str):
        nums = re.findall(r"\d+", v)
        return [int(x) for x in nums] or [0]

    lines = []
    prev = None
    order = sorted(nodes, key=key)
    for i, node in enumerate(order):
        body = " ".join(f"{f};" for f in nodes[node])
        if i == 0:
            body += f" {extra_global}"
        tail = f" {prev};" if prev else ";"
        if i == len(order) - 1:
            lines.append(f"{node} {{ global: {body} local: *; }}{tail}")
        else:
            lines.append(f"{node} {{ global: {body} }}{tail}")
        prev = node
    return "\n".join(lines) + "\n"


def build_fakes(force: bool = False) -> dict[str, Path]:
    FAKES_OUT.mkdir(parents=True, exist_ok=True)
    res: dict[str, Path] = {}
    versions = _hip_versions()

    hsa_src = NATIVE / "fakes" / "fake_hsa.cpp"
    hsa = FAKES_OUT / "libhsa-runtime64.so.1"
    if force or not _stamp(hsa, [hsa_src]):
        vs = FAKES_OUT / "hsa.map"
        vs.write_text(_version_script(hsa_src, "ROCR_1", {}, "fake_hsa_queue_count; fake_hsa_queue_mask; fake_hsa_pool_used; fake_hsa_tools_loaded; open; hsa_signal_wait_scacquire; fake_hsa_submit; fake_hsa_dispatched; fake_hsa_intercept_queues;"))
        _run([CXX, *COMMON, hsa_src, "-o", hsa, "-shared", "-Wl,-soname,libhsa-runtime64.so.1",
              f"-Wl,--version-script={vs}", "-lpthread"])
        _mark(hsa, [hsa_src])
    res["hsa"] = hsa

    hip_src = NATIVE / "fakes" / "fake_hip.cpp"
    hip = FAKES_OUT / "libamdhip64.so.7"
    hip_extra = ("fake_hip_launches; fake_hip_launch_blocks; fake_hip_physical_used; fake_hip_graph_create; "
                 "fake_hip_exec_ns; fake_hip_svm_move; fake_hip_managed_gpu_bytes; fake_hip_host_touch_bytes; fake_hip_memsets; fake_hip_prefetch_overflows; fake_hip_peer_copies; "
                 "fake_hip_branchy_single_queue_launches; fake_hip_exec_graph; "
                 "_Z24hipExtModuleLaunchKernelP18ihipModuleSymbol_tjjjjjjmP12ihipStream_tPPvS4_P11ihipEvent_tS6_j; "
                 "_Z24hipHccModuleLaunchKernelP18ihipModuleSymbol_tjjjjjjmP12ihipStream_tPPvS4_P11ihipEvent_tS6_;")
    if force or not _stamp(hip, [hip_src, hsa_src], hip_extra + str(sorted(versions.items()))[:4096]):
        vs = FAKES_OUT / "hip.map"
        vs.write_text(_version_script(hip_src, "hip_4.2", versions, hip_extra))
        _run([CXX, *COMMON, hip_src, "-o", hip, "-shared", "-Wl,-soname,libamdhip64.so.7",
              f"-Wl,--version-script={vs}", f"-L{FAKES_OUT}", "-l:libhsa-runtime64.so.1",
              f"-Wl,-rpath,{FAKES_OUT}", "-ldl", "-lpthread"])
        _mark(hip, [hip_src, hsa_src], hip_extra + str(sorted(versions.items()))[:4096])
    res["hip"] = hip

    smi_src = NATIVE / "fakes" / "fake_amdsmi.cpp"
    if smi_src.exists():
        smi = FAKES_OUT / "libamd_smi.so"
        if force or not _stamp(smi, [smi_src]):
            _run([CXX, *COMMON, smi_src, "-o", smi, "-shared", "-Wl,-soname,libamd_smi.so",
                  "-lpthread"])
            _mark(smi, [smi_src])
        res["smi"] = smi

    rsmi_src = NATIVE / "fakes" / "fake_rsmi.cpp"
    if rsmi_src.exists():
        rsmi = FAKES_OUT / "librocm_smi64.so.1"
        if force or not _stamp(rsmi, [rsmi_src]):
            _run([CXX, *COMMON, rsmi_src, "-o", rsmi, "-shared", "-Wl,-soname,librocm_smi64.so.1"])
            _mark(rsmi, [rsmi_src])
        res["rsmi"] = rsmi

    rccl_src = NATIVE / "fakes" / "fake_rccl.cpp"
    if rccl_src.exists():
        rccl = FAKES_OUT / "librccl_fake.so"
        if force or not _stamp(rccl, [rccl_src]):
            _run([CXX, *COMMON, rccl_src, "-o", rccl, "-shared"])
            _mark(rccl, [rccl_src])
        res["rccl"] = rccl

    scope_src = NATIVE / "fakes" / "fake_scope.cpp"
    if scope_src.exists():
        dep, user = FAKES_OUT / "libscope_dep.so", FAKES_OUT / "libscope_user.so"
        if force or not _stamp(user, [scope_src]):
            _run([CXX, *COMMON, "-DSCOPE_DEP", scope_src, "-o", dep, "-shared", "-Wl,-soname,libscope_dep.so"])
            _run([CXX, *COMMON, scope_src, "-o", user, "-shared", f"-L{FAKES_OUT}", "-l:libscope_dep.so",
                  f"-Wl,-rpath,{FAKES_OUT}", "-ldl"])
            _mark(user, [scope_src])
        res["scope"] = user

    drv_src = NATIVE / "tests" / "shim_driver.cpp"
    drv = FAKES_OUT / "shim_driver"
    if force or not _stamp(drv, [drv_src, hip_src, hsa_src] + _headers()):
        _run([CXX, *COMMON, "-Wno-unused-result", drv_src, "-o", drv, f"-L{FAKES_OUT}", "-l:libamdhip64.so.7",
              "-l:libhsa-runtime64.so.1", f"-Wl,-rpath,{FAKES_OUT}", "-ldl", "-lpthread"])
        _mark(drv, [drv_src, hip_src, hsa_src] + _headers())
    res["driver"] = drv
    return res


def have_hipcc() -> bool:
    return Path(HIPCC).exists()


def build_all(sanitize: str | None = None, kernels: bool = True) -> dict[str, Path]:
    out = {"shim": build_shim(), "fakes": build_fakes(), "sched": build_sched()}
    if (NATIVE / "smi").exists() and any((NATIVE / "smi").glob("*.cpp")):
        out["smi"] = build_smi()
    if sanitize:
        out["shim_" + sanitize] = build_shim(sanitize)
    if kernels and have_hipcc() and any((NATIVE / "kernels").glob("*.hip")):
        out["kernels"] = build_kernels()
        out["probe_module"] = build_probe_module()
    return out


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("targets", nargs="*", default=["all"])
    ap.add_argument("--sanitize", choices=["thread", "address"], default=None)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    for t in a.targets:
        if t == "all":
            build_all(a.sanitize)
        elif t == "shim":
            build_shim(a.sanitize, a.force)
        elif t == "fakes":
            build_fakes(a.force)
        elif t == "kernels":
            build_kernels(a.force)
        elif t == "smi":
            build_smi(a.force)
        elif t == "sched":
            build_sched(a.force)
        elif t == "clean":
            shutil.rmtree(OUT, ignore_errors=True)
        else:
            print(f"unknown target {t}", file=sys.stderr)
            return 2
    return 0


if __name__ == "__main__":
    sys.exit(main())
