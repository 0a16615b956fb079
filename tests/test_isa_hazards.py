"""The product library's gfx950 machine code is free of the VMEM store-data hazard that corrupted
the reverted per-utterance-descriptor streaming kernel: no VALU overwrites a
data VGPR of a >64-bit vector store within 2 wait states of it. LLVM skips those wait states for
buffer stores with a register soffset, so this is checked on the built code, not assumed.
CPU only (llvm-objdump of the embedded code objects)."""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
import isa_hazards as H  # noqa: E402


# the instruction pair found in the study build's k_fwd_bwd_stream (make lib-var-desc): the
# v_cndmask that materialises a boolean lands in the first data VGPR of the gradient store
HAZARD = """
_Z1kv:
\tbuffer_store_dwordx4 v[28:31], v77, s[40:43], s14 offen
\tv_cndmask_b32_e64 v28, 0, 1, s[66:67]
\ts_endpgm
"""


def _scan_text(tmp_path, text):
    f = tmp_path / "k.s"
    f.write_text(text)
    return H.scan(H.parse(H.disassemble(f)))


def test_scanner_flags_the_study_build_pattern(tmp_path):
    bad = _scan_text(tmp_path, HAZARD)
    assert len(bad) == 1 and "v_cndmask_b32_e64 v28" in bad[0]


def test_scanner_accepts_two_wait_states(tmp_path):
    ok = HAZARD.replace("s14 offen\n", "s14 offen\n\ts_nop 1\n")
    assert _scan_text(tmp_path, ok) == []
    one = HAZARD.replace("s14 offen\n", "s14 offen\n\ts_nop 0\n")  # 1 wait state: not enough
    assert len(_scan_text(tmp_path, one)) == 1
    other = HAZARD.replace("v_cndmask_b32_e64 v28", "v_cndmask_b32_e64 v32")  # not store data
    assert _scan_text(tmp_path, other) == []


def test_scanner_follows_the_fall_through_of_a_conditional_branch(tmp_path):
    # a not-taken s_cbranch continues the straight-line window
    ft = HAZARD.replace("s14 offen\n", "s14 offen\n\ts_cbranch_scc0 .LBB0_1\n") + ".LBB0_1:\n\ts_endpgm\n"
    bad = _scan_text(tmp_path, ft)
    assert len(bad) == 1 and "after 1 wait state" in bad[0]
    # an unconditional branch ends the straight-line path; its target is checked in taken mode
    br = HAZARD.replace("s14 offen\n\tv_cndmask_b32_e64 v28, 0, 1, s[66:67]\n",
                        "s14 offen\n\ts_branch .LBB0_1\n\ts_endpgm\n.LBB0_1:\n"
                        "\tv_cndmask_b32_e64 v28, 0, 1, s[66:67]\n")
    f = tmp_path / "b.s"
    f.write_text(br)
    insts = H.parse(H.disassemble(f))
    assert H.scan(insts) == []
    assert len(H.scan(insts, taken=True)) == 1
    # EXEC unchanged since the store: a taken s_cbranch_execz means the store wrote nothing
    ez = br.replace("s_branch .LBB0_1", "s_cbranch_execz .LBB0_1")
    f.write_text(ez)
    assert H.scan(H.parse(H.disassemble(f)), taken=True) == []


@pytest.mark.parametrize("lib", ["libssnt_tts_c.so", "ab/libssnt_tts_c_ab.so"])
def test_built_libraries_have_no_straight_line_store_data_hazard(lib):
    # the product library, and the A/B library the forced-kernel parity cases run through
    path = ROOT / "ssnt-tts-rust_amd" / "lib" / lib
    if not path.exists():
        pytest.fail(f"build the library first (make lib lib-ab): {path}")
    insts = H.parse(H.disassemble(path))
    stores = sum(1 for mn, *_ in insts if H._WIDE_STORE.match(mn))
    assert stores > 100  # the fwd-bwd kernels' 16-byte gradient / row stores are in the scan
    bad = H.scan(insts)
    assert not bad, "\n".join(bad[:10])
