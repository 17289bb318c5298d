#!/usr/bin/env python3
"""Configure + build the native engine (CMake/Ninja, ROCm clang, --offload-arch=gfx950).

    python build.py            # incremental build into ./build, libs into the Python package
    python build.py --clean    # from scratch
    python build.py --sanitize address   # host-only sanitizer build in ./build-asan
"""
import argparse
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def build(clean=False, jobs=None, sanitize="", build_dir=None, verbose=False):
    bdir = build_dir or os.path.join(ROOT, "build" if not sanitize else f"build-{sanitize}")
    if clean and os.path.isdir(bdir):
        shutil.rmtree(bdir)
    os.makedirs(bdir, exist_ok=True)
    cxx = os.path.join(ROCM, "llvm", "bin", "clang++")
    cfg = ["cmake", "-G", "Ninja", "-S", ROOT, "-B", bdir, f"-DCMAKE_CXX_COMPILER={cxx}",
           f"-DROCM_PATH={ROCM}", f"-DPython3_EXECUTABLE={sys.executable}", "-DCMAKE_BUILD_TYPE=Release"]
    if sanitize:
        cfg += [f"-DNM03_SANITIZE={sanitize}",
                f"-DNM03_PY_OUT={os.path.join(bdir, 'lib')}"]
    if not os.path.exists(os.path.join(bdir, "build.ninja")):
        subprocess.run(cfg, check=True, stdout=None if verbose else subprocess.DEVNULL)
    jobs = jobs or min(16, os.cpu_count() or 4)
    cmd = ["cmake", "--build", bdir, "-j", str(jobs)]
    subprocess.run(cmd, check=True)
    return bdir


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", "--jobs", type=int)
    ap.add_argument("--sanitize", default="")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    build(a.clean, a.jobs, a.sanitize, verbose=a.verbose)


if __name__ == "__main__":
    main()
