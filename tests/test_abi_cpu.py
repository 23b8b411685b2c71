"""The C ABI boundary without a GPU: libttamm.so loads, exports every entry point that
include/ttamm.h declares, the ctypes mirror covers them all, and the ctypes struct layouts
equal what a C compiler (gcc) produces for the header."""

import ctypes
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "ttamm.h"


def header_functions() -> list[str]:
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ttamm_[a-z0-9_]+)\s*\(", text)))


def test_header_parses_as_c_and_cxx(tmp_path):
    from ttamm import _lib

    src = tmp_path / "h.c"
    src.write_text(f'#include "{HEADER}"\nint main(void) {{ return TTAMM_ABI_VERSION == {_lib.ABI_VERSION} ? 0 : 1; }}\n')
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", str(src), "-o", str(tmp_path / "h")], check=True)
    subprocess.run([str(tmp_path / "h")], check=True)
    cxx = tmp_path / "h.cpp"
    cxx.write_text(src.read_text())
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", str(cxx), "-o", str(tmp_path / "hx")], check=True)


def test_library_exports_every_declared_function():
    from ttamm import _lib

    lib = _lib.load()
    declared = header_functions()
    assert declared, "no functions parsed from the header"
    assert sorted(_lib.SIGNATURES) == declared
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.library_path())], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (ttamm_\w+)", out))
    assert set(declared) <= exported, sorted(set(declared) - exported)
    for name in declared:
        assert hasattr(lib, name)
    assert lib.ttamm_abi_version() == _lib.ABI_VERSION
    assert lib.ttamm_last_error() is not None


STRUCTS = {
    "ttamm_linear": "Linear",
    "ttamm_table": "Table",
    "ttamm_tower": "Tower",
    "ttamm_hparams": "HParams",
    "ttamm_batch": "Batch",
    "ttamm_step_args": "StepArgs",
}


def test_ctypes_layout_matches_c(tmp_path):
    from ttamm import _lib

    lines = [f'#include "{HEADER}"', "#include <stdio.h>", "#include <stddef.h>", "int main(void) {"]
    for cname, pyname in STRUCTS.items():
        cls = getattr(_lib, pyname)
        lines.append(f'printf("{pyname} size %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            lines.append(f'printf("{pyname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", str(src), "-o", str(exe)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                              check=True).stdout.splitlines())
    for cname, pyname in STRUCTS.items():
        cls = getattr(_lib, pyname)
        assert int(got[f"{pyname} size"]) == ctypes.sizeof(cls), pyname
        for fname, _ in cls._fields_:
            assert int(got[f"{pyname}.{fname}"]) == getattr(cls, fname).offset, f"{pyname}.{fname}"


def test_errors_map_to_reference_exceptions():
    """Invalid arguments come back as TTAMM_E_INVALID -> ValueError, with no device work."""
    from ttamm import _lib

    lib = _lib.load()
    with pytest.raises(ValueError):
        _lib.check(lib.ttamm_gather_rows(None, 10, 0, None, 5, None, 0, None))
    with pytest.raises(ValueError):
        _lib.check(lib.ttamm_sample_negatives(None, 4, 0, 10, None, None, 0, 0, 0, 0, None, None, None))
    # (non-null placeholders: the argument checks fail before any device access)
    with pytest.raises(ValueError, match="num_items must be greater than one"):
        _lib.check(lib.ttamm_sample_negatives(8, 4, 2, 1, None, None, 0, 0, 0, 0, 8, 8, None))
    with pytest.raises(ValueError, match="num_negatives"):
        _lib.check(lib.ttamm_sample_negatives(8, 4, 0, 10, None, None, 0, 0, 0, 0, 8, 8, None))
    with pytest.raises(ValueError):
        _lib.check(lib.ttamm_check_rows(None, 4, 10, None, 0, 0, 8, None))
    with pytest.raises(ValueError):
        _lib.check(lib.ttamm_adamw_dense(None, None, None, None, 4, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1, 0, None))
    with pytest.raises(ValueError):
        _lib.check(lib.ttamm_train_step(None, None))


def test_train_step_validation_rejects_bad_descriptors():
    """The executor validates the reference's shape constraints before touching the GPU."""
    from ttamm import _lib

    lib = _lib.load()
    args = _lib.StepArgs()
    with pytest.raises(ValueError, match="embedding table"):
        _lib.check(lib.ttamm_train_step(ctypes.byref(args), None))
    fake = 4096  # never dereferenced: validation fails first
    for tower in (args.user, args.item):
        tower.id.weight = tower.id.exp_avg = tower.id.exp_avg_sq = fake
        tower.id.rows = 10
        tower.id.dim = 6
    with pytest.raises(ValueError, match="% 4"):
        _lib.check(lib.ttamm_train_step(ctypes.byref(args), None))
    assert lib.ttamm_train_step_workspace_size(ctypes.byref(args)) > 0


@pytest.mark.parametrize("row_base", [-1, 5])
def test_inbatch_bce_rejects_row_base_outside_the_columns(row_base):
    """ttamm_inbatch_bce checks row_base itself (not only the Python wrapper): the B users' label
    diagonal must lie inside the Bc positive columns.  The check runs before any device work, so
    it is exercised here with host buffers that are never touched."""
    from ttamm import _lib

    lib = _lib.load()
    B, Bc, D = 4, 8, 16
    buf = (ctypes.c_float * 64)()
    loss = ctypes.c_double(0.0)
    ws = (ctypes.c_char * 16)()
    p = ctypes.cast(buf, ctypes.c_void_p)
    rc = lib.ttamm_inbatch_bce(p, B, D, p, Bc, D, D, row_base, 1.0, p, D, p, D, ctypes.byref(loss),
                               ctypes.cast(ws, ctypes.c_void_p), 16, None)
    assert rc != 0
    assert b"row_base" in lib.ttamm_last_error()


@pytest.mark.parametrize("case,want", [
    ("fp32-d96", 1), ("fp32-d32", 1), ("fp32-d8-generic", 0), ("no-mimic", 0), ("bf16-d128", 1),
    ("bf16-d64", 0), ("user-hg-differs", 0), ("item-sum-fusion", 0),
])
def test_exchange_compact_supported_is_host_logic(case, want):
    """ttamm_exchange_compact_supported (host only, no device call): compact exchange rows need
    mimic, a gated item tower, and the fused gate kernels for it alone and grouped with the user
    tower — gate.hip at D = Hg in {32, 64, 96, 128} (fp32), gate16.hip at D = Hg in {128, 256}
    (bf16); anything else keeps the 2D-wide rows."""
    from ttamm import _lib

    lib = _lib.load()
    a = _lib.StepArgs()
    D = {"fp32-d32": 32, "fp32-d8-generic": 8, "bf16-d128": 128, "bf16-d64": 64}.get(case, 96)
    bf = 1 if case.startswith("bf16") else 0
    for t in (a.user, a.item):
        t.id.dim = D
        t.fusion = 2  # TTAMM_FUSION_GATED
        t.gate[0].out_features = D
        t.gate[0].in_features = 2 * D
        t.gate[1].out_features = D
        t.gate[1].in_features = D
        t.matmul_bf16 = bf
    a.mimic_enabled = 0 if case == "no-mimic" else 1
    if case == "user-hg-differs":
        a.user.gate[0].out_features = 64
    if case == "item-sum-fusion":
        a.item.fusion = 1  # TTAMM_FUSION_SUM
    assert lib.ttamm_exchange_compact_supported(ctypes.byref(a)) == want


# The documented environment knobs (INTEGRATION.md "Environment"); every other TTAMM_* switch in
# the sources is a developer A/B / ablation / measured-slower variant read only by a `make DEV=1`
# library (csrc/common.h dev_env).  TTAMM_DENSE_* / TTAMM_G0_* are enum names in error messages.
DOCUMENTED_ENV = {"TTAMM_FP32_MFMA", "TTAMM_RETRIEVAL_FP32", "TTAMM_GENERIC_GATE"}
ENUM_NAMES = {"TTAMM_DENSE_ADAM", "TTAMM_DENSE_SGD", "TTAMM_G0_EXACT", "TTAMM_G0_FAST"}
DEV_SWITCHES = ("TTAMM_GATE_ABLATE", "TTAMM_RETRIEVAL_ABLATE", "TTAMM_BF16_WGRAD256", "TTAMM_PROLOGUE_PREP",
                "TTAMM_SLICE_LATE", "TTAMM_GATE16_SPLIT", "TTAMM_WGRAD_ROWS_PER_SPLIT", "TTAMM_FEATURE_PLANES")


def test_default_library_reads_only_documented_env_knobs():
    """the default build names no developer switch at all — the getenv calls
    behind them are compiled out (dev_env returns nullptr), so a stray ablation variable in a
    user's environment cannot change what the drop-in library computes."""
    from ttamm import _lib

    lib = _lib.load()
    assert lib.ttamm_developer_build() == 0
    blob = _lib.library_path().read_bytes()
    names = {m.decode() for m in re.findall(rb"TTAMM_[A-Z0-9_]+", blob)}
    assert names - ENUM_NAMES <= DOCUMENTED_ENV, sorted(names - ENUM_NAMES - DOCUMENTED_ENV)
    for name in DEV_SWITCHES:
        assert name not in names
    # the Python host reads only TTAMM_WIDE_EXCHANGE (documented) and TTAMM_LIBRARY (the loader)
    pkg = ROOT / "two-tower-augmented-with-adaptive-mimic-mechanism_amd" / "ttamm"
    env_reads = set()
    for f in pkg.glob("*.py"):
        env_reads |= set(re.findall(r"os\.environ(?:\.get)?\(?\[?\"(TTAMM_[A-Z0-9_]+)", f.read_text()))
    assert env_reads <= {"TTAMM_WIDE_EXCHANGE", "TTAMM_LIBRARY"}, env_reads
