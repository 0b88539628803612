"""Python mirror of csum_api.cpp xwalk_auto: the fixed-stride dispatch table the library compiles in
(smoltcp_amd/csrc/dispatch_table.inc), read from the same file, so that the tests know which kernel
and variant a batch should run without restating the table."""
import os
import re

_INC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "smoltcp_amd", "csrc",
                    "dispatch_table.inc")


def _tables():
    text = open(_INC).read()
    out = {}
    for name in ("kVerifyTable", "kEmitTable"):
        body = text.split(name, 1)[1].split("};", 1)[0]
        out[name] = re.findall(r'"([a-z]{3})"', body)
        assert len(out[name]) == 125, name
    return out


TABLES = _tables()


def fixed_variant(op: str, length: int, stride: int) -> int:
    """The variant xwalk_auto picks for a fixed-stride batch ("emit" / "verify"); 0: the walk kernel
    (whose own default is then 39 for emit, 5 for verify)."""
    if stride < length or length < 1024 or length >= 1024 + 64 * 125:
        return 0
    k = (length - 1024) // 64
    col = 2 if stride != length else (0 if length % 64 == 0 else 1)
    c = TABLES["kVerifyTable" if op == "verify" else "kEmitTable"][k][col]
    if op == "verify":
        return {"h": 89, "x": 47, "w": 0}[c]
    return {"t": 101, "n": 57, "x": 47, "w": 0}[c]


def fixed_launch(op: str, length: int, stride: int):
    """(kernel, variant) the default dispatch launches for a fixed-stride KIND_IP batch."""
    v = fixed_variant(op, length, stride)
    if v:
        return "xwalk_kernel", v
    return "csum_kernel", 39 if op == "emit" else 5
