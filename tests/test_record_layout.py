"""The ragged parameter records' slot layout is defined twice -- the device header
(csrc/hip/params.h) and the host's encoder (models/kinetics.py) -- and they must agree."""
import re
from pathlib import Path

from magicsoup_amd.models import kinetics as K

_HDR = Path(__file__).resolve().parents[1] / "magicsoup_amd" / "csrc" / "hip" / "params.h"


def _const(name: str) -> int:
    m = re.search(rf"constexpr int {name} = ([^;]+);", _HDR.read_text())
    assert m, name
    return int(eval(m.group(1), {"__builtins__": {}}))  # (integer literals and shifts only)


def test_slot_fields_match_the_device_header():
    assert _const("kRecOffBits") == K._REC_OFF_BITS
    assert _const("kRecCntBits") == K._REC_CNT_BITS
    assert _const("kRecMaxProteins") == K._MAX_PROTEINS


def test_slot_code_round_trip_past_8191_proteins():
    for off, cnt, width in ((0, 1, 1), (123456789, 9282, 14418), ((1 << 32) - 1, K._MAX_PROTEINS, K._MAX_PROTEINS)):
        v = K._rec_code(off, cnt, width)
        assert 0 <= v < (1 << 63)  # (the sign bit stays clear)
        assert v & ((1 << K._REC_OFF_BITS) - 1) == off
        assert (v >> K._REC_OFF_BITS) & K._REC_CNT_MASK == cnt
        assert v >> (K._REC_OFF_BITS + K._REC_CNT_BITS) == width
