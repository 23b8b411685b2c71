"""The built code objects hold no packed-FP32 instruction whose high half reads the
destination's low register (tools/check_pk_operands.py: such an instruction made the fast g = 0
replay's results timing-dependent on MI355X), and the checker recognises the pattern."""

from __future__ import annotations

import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
import check_pk_operands as chk  # noqa: E402

BUILD = ROOT / "two-tower-augmented-with-adaptive-mimic-mechanism_amd" / "build"


def test_checker_flags_high_half_reading_destination_low():
    listing = [
        "0000000000001000 <k>:",
        # the replay's instruction: src1 broadcast from v48 (op_sel_hi 0), destination v[48:49]
        "\tv_pk_fma_f32 v[48:49], v[54:55], v[48:49], v[48:49] op_sel:[0,0,1] op_sel_hi:[1,0,1]// 00: 0",
        # lane-aligned overlap: each half reads its own register
        "\tv_pk_fma_f32 v[52:53], v[56:57], v[52:53], v[54:55]// 00: 0",
        # broadcast from a register the destination does not overlap
        "\tv_pk_mul_f32 v[20:21], v[24:25], v[20:21] op_sel_hi:[0,1]// 00: 0",
        # a source pair one below the destination: its high register is the destination's low
        "\tv_pk_add_f32 v[10:11], v[9:10], v[12:13]// 00: 0",
    ]
    got = chk.hazards_in_listing(listing)
    assert [f for f, _ in got] == ["k", "k"]
    assert "v[54:55], v[48:49]" in got[0][1] and "v[9:10]" in got[1][1]


def test_built_objects_are_clean():
    objs = sorted(BUILD.glob("*.o"))
    if not objs:
        pytest.skip("library not built")
    bad, empty = [], []
    for o in objs:
        hazards, nfunc = chk.scan_object(o)
        bad += [(o.name, f, i) for f, i in hazards]
        if nfunc == 0 and o.name in chk.KERNEL_OBJECTS:
            empty.append(o.name)
    assert not bad, bad[:5]
    # the scan must see every kernel object's device code (a toolchain change in the fat-binary
    # section or bundle name would otherwise make it check nothing)
    assert not empty, empty
