"""Register budget of the lane-walk tile kernels (CPU: hipcc cross-compiles gfx950 assembly).

The tile kernel's LDS plan allows 4 workgroups of 256 threads per CU, i.e. 4 waves per SIMD, so each
K bucket may use up to 128 VGPRs without losing occupancy. A source change that looks neutral can
push a bucket over it (round 6: an own-row split with two inlined copies of the scan loop took the
K=50 bucket from 119 to 177 VGPRs -- 2 waves per SIMD, +30 % query time -- and the K=64 bucket from
13 to 82 spilled VGPRs). This test pins the budget: every lane-walk bucket <= 128 VGPRs, no spills
up to K=50, and at most a handful at K=64 (its waves-per-EU cap trades a few spills for occupancy).
"""
import re
import subprocess

import pytest

from cuda_knearests_amd import _build

pytestmark = pytest.mark.slow


def _metadata(tmp_path):
    out = tmp_path / "query.s"
    cmd = [_build.HIPCC] + _build.HIPFLAGS + ["--cuda-device-only", "-S", str(_build.CSRC / "kernels/query.hip"),
                                                "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    res = {}
    for blk in out.read_text().split("- .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        m = re.search(r"knn_tile_kernelILi(\d+)ELi\d+ELb1ELb0E", name)
        if not m:
            continue
        res[int(m.group(1))] = (int(re.search(r"\.vgpr_count:\s+(\d+)", blk).group(1)),
                                int(re.search(r"\.vgpr_spill_count:\s+(\d+)", blk).group(1)))
    return res


def test_lane_walk_register_budget(tmp_path):
    res = _metadata(tmp_path)
    assert {4, 8, 16, 32, 50, 64} <= set(res), res
    for k, (vgpr, spill) in sorted(res.items()):
        assert vgpr <= 128, (k, vgpr)
        assert spill == 0 or (k > 50 and spill <= 24), (k, spill)
