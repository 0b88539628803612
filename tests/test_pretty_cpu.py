"""The pretty-print / partial-checksum path: checksum::format_checksum
(src/wire/ip.rs:871-886) as the packet listings use it — the IPv4 line (ipv4.rs:698) and the
UDP / TCP line (pretty_print_ip_payload, ip.rs:930-962) — computed from a verify status byte.
Pinned by the module example of src/wire/pretty_print.rs (an IPv4 header whose checksum is wrong:
"(checksum incorrect)") and by the fuzz-corpus frames that carry TX-offload partial checksums."""
import numpy as np

import oracle
from smoltcp_amd import checksum

KIND_ETH = 2


def test_format_checksum():
    assert checksum.format_checksum(True, False) == ""
    assert checksum.format_checksum(True, True) == ""
    assert checksum.format_checksum(False, True) == " (partial checksum correct)"
    assert checksum.format_checksum(False, False) == " (checksum incorrect)"


def test_pretty_print_example(golden):
    ex = golden["pretty_print"][0]
    frame = np.frombuffer(bytes.fromhex(ex["bytes"]), np.uint8).copy()
    st = oracle.batch_verify(frame, None, 1, len(frame), len(frame), KIND_ETH)[0]
    assert checksum.ipv4_annotation(int(st)) == ex["ipv4_annotation"] == " (checksum incorrect)"


def test_corpus_partial_checksums(golden):
    """tcpv4_data / tcpv4_fin / tcpv4_syn carry partial (pseudo-header-only) checksums: their TCP
    line reads "(partial checksum correct)"; the frames with full checksums read nothing."""
    for f in golden["fuzz_corpus_frames"]:
        frame = np.frombuffer(bytes.fromhex(f["bytes"]), np.uint8).copy()
        st = int(oracle.batch_verify(frame, None, 1, len(frame), len(frame), KIND_ETH)[0])
        assert checksum.ipv4_annotation(st) == "", f["name"]
        want = " (partial checksum correct)" if f["name"] in ("tcpv4_data.bin", "tcpv4_fin.bin", "tcpv4_syn.bin") else ""
        assert checksum.l4_annotation(st) == want, f["name"]
