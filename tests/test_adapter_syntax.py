"""The reference-side adapter compiles (SURVEY.md §8 f1 / INTEGRATION.md §4).

adapter/hipOptimizer.cc (the source a maintainer adds to the reference tree)
and adapter/Optimizer_hip_dispatch.cc (the Optimizer.cc dispatch that selects
it, include/backend/Optimizer.h:42-71 + HIP) go through `g++ -fsyntax-only`
against declaration-only stand-ins of the reference headers they include
(tests/adapter_syntax/: KeyFrame, MapPoint, Map, LoopClosing, Converter,
lidarConfig, g2oOptimizer, g2o::Sim3, and the cv::Mat / PCL / Eigen members
used), laid out as the reference's include directories
(CMakeLists.txt:103-115). The stand-ins carry the reference's signatures, so
a type or declaration error in the adapter fails here; nothing is linked.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUBS = os.path.join(ROOT, "tests", "adapter_syntax")
INCLUDES = ["", "data_structure", "utils", "backend"]


def _compile(src):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    cmd = [cxx, "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror"]
    cmd += ["-I" + os.path.join(STUBS, d) for d in INCLUDES] + ["-I" + os.path.join(ROOT, "include")]
    cmd.append(os.path.join(ROOT, "adapter", src))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr


@pytest.mark.parametrize("src", ["hipOptimizer.cc", "Optimizer_hip_dispatch.cc"])
def test_adapter_compiles_against_reference_declarations(src):
    _compile(src)
