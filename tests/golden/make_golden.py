#!/usr/bin/env python3
"""Generate tests/golden/kat.json from the reference's own test vectors.

Run in the build container (the only place /root/reference exists):

    python tests/golden/make_golden.py [/root/reference]

It reads the reference's Rust test modules as TEXT, extracts the known-answer byte arrays by name
(and the inline IPv6 packets of src/iface/interface/tests/ipv6.rs whose tests assert that
``parse_ipv6`` — ICMPv6 checksum verified with default caps — succeeds), and copies the fuzz-corpus
frames.  The expected checksum values and the pre-fill field contents are the ones the reference
tests assert / set up; each entry cites the file:line it comes from.  Nothing from the reference is
executed (there is no Rust toolchain here).  The output is data only: input bytes + expected
results.
"""
from __future__ import annotations

import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat.json")


def _read(rel):
    with open(os.path.join(REF, rel)) as f:
        return f.read()


def _parse_array(body: str) -> bytes:
    toks = [t.strip() for t in body.replace("\n", " ").split(",")]
    return bytes(int(t, 0) for t in toks if t)


def static_array(rel: str, name: str):
    """Return (bytes, line) of ``static NAME: [u8; N] = [ ... ];`` in file ``rel``."""
    text = _read(rel)
    m = re.search(r"static\s+%s\s*:\s*\[u8;\s*(\d+)\]\s*=\s*\[(.*?)\];" % re.escape(name), text,
                  re.S)
    if not m:
        raise SystemExit(f"{rel}: array {name} not found")
    b = _parse_array(m.group(2))
    assert len(b) == int(m.group(1)), (rel, name)
    return b, text[: m.start()].count("\n") + 1


def inline_ipv6_packets(rel: str):
    """Inline ``let data = [..];`` arrays whose test asserts ``parse_ipv6(&data)`` is ``Ok``."""
    text = _read(rel)
    out = []
    for m in re.finditer(r"let data = \[(.*?)\];", text, re.S):
        tail = text[m.end(): m.end() + 200]
        if re.match(r"\s*assert_eq!\(\s*parse_ipv6\(&data\),\s*Ok\(", tail):
            out.append((_parse_array(m.group(1)), text[: m.start()].count("\n") + 1))
    return out


def hop_by_hop_packets(rel: str):
    """The IPv6 packets with a Hop-by-Hop header of the ``hop_by_hop_*`` iface tests, with the
    response each test asserts for ``process_ipv6``: ``None`` (dropped silently), an ICMPv6
    ParamProblem (dropped, with an error reply) or an EchoReply (accepted: the ICMPv6 echo request
    behind the header passed its checksum gate)."""
    text = _read(rel)
    out = []
    for m in re.finditer(r"fn (hop_by_hop_\w+)\(", text):
        body_end = text.find("\n}\n", m.end())
        body = text[m.end(): body_end]
        d = re.search(r"let data = \[(.*?)\];", body, re.S)
        r = re.search(r"let response = (None|Some\(.*?IpPayload::Icmpv6\(Icmpv6Repr::(\w+))", body, re.S)
        if not d or not r:
            raise SystemExit(f"{rel}: {m.group(1)} has no data / response")
        resp = "None" if r.group(1) == "None" else r.group(2)
        line = text[: m.end() + d.start()].count("\n") + 1
        out.append({"name": m.group(1), "kind": "ip", "bytes": _parse_array(d.group(1)).hex(),
                    "response": resp, "dropped": resp != "EchoReply",
                    "cite": f"{rel}:{line} ({m.group(1)}: process_ipv6 returns {resp})"})
    return out


V4_A = "c0a80101"  # 192.168.1.1 (udp.rs:373, tcp.rs:1240)
V4_B = "c0a80102"  # 192.168.1.2
FE80_1 = "fe800000000000000000000000000001"  # icmpv6.rs:851, ndisc.rs:466
FE80_2 = "fe800000000000000000000000000002"
FF02_1 = "ff020000000000000000000000000001"  # IPV6_LINK_LOCAL_ALL_NODES (mld.rs construct)
FF02_2 = "ff020000000000000000000000000002"  # IPV6_LINK_LOCAL_ALL_ROUTERS


def _eui64_iid(ext_le: bytes) -> bytes:
    """IPv6 interface identifier of an IEEE 802.15.4 extended address as it sits in the frame
    (little-endian): reverse the bytes, flip the universal/local bit (RFC 4944 §6)."""
    ext = ext_le[::-1]
    return bytes([ext[0] ^ 0x02]) + ext[1:]


def sixlowpan_nhc_udp():
    """The 6LoWPAN NHC UDP datagram of test sixlowpan_three_fragments (src/wire/sixlowpan/mod.rs):
    three IEEE 802.15.4 frames (2003 frame, PAN-ID compression, extended addresses: 21-byte MAC
    header), FRAG1 (4 bytes) + IPHC 0x6e33 (TF=01: 3 bytes inline, NH compressed, HLIM elided,
    SAM=DAM=11: addresses from the link-layer addresses) + NHC UDP, then two FRAGN (5 bytes).  The
    reassembled NHC UDP packet and its link-local addresses; its inline checksum 0xb46b is what
    UdpNhcRepr::parse (nhc.rs:697-723) checks under caps.udp.rx().  (The datagram of
    src/iface/interface/tests/sixlowpan.rs test_sixlowpan_udp_with_fragmentation is not used: that
    test disables UDP checksums and its inline checksum does not match its payload.)"""
    rel = "src/wire/sixlowpan/mod.rs"
    text = _read(rel)
    frames, lines = [], []
    for name in ("frame1", "frame2", "frame3"):
        m = re.search(r"let %s: &\[u8\] = &\[(.*?)\];" % name, text, re.S)
        if not m:
            raise SystemExit(f"{rel}: {name} not found")
        frames.append(_parse_array(m.group(1)))
        lines.append(text[: m.start()].count("\n") + 1)
    mac = 21
    f1, f2, f3 = frames
    assert f1[mac] >> 3 == 0x18 and f2[mac] >> 3 == 0x1C and f3[mac] >> 3 == 0x1C  # FRAG1 / FRAGN
    iphc = f1[mac + 4:]
    assert iphc[0] == 0x6E and iphc[1] == 0x33
    nhc = iphc[2 + 3:]  # TF=01 carries 3 bytes
    assert nhc[0] >> 3 == 0x1E and nhc[0] & 7 == 0  # UDP, checksum inline, both ports inline
    pkt = nhc + f2[mac + 5:] + f3[mac + 5:]
    size = (f1[mac] & 7) << 8 | f1[mac + 1]  # datagram_size (uncompressed IPv6 + UDP + payload)
    assert len(pkt) - 7 == size - 48
    dst_le, src_le = f1[5:13], f1[13:21]
    return [{
        "name": "sixlowpan_three_fragments_udp",
        "bytes": pkt.hex(),
        "src": (bytes.fromhex("fe80000000000000") + _eui64_iid(src_le)).hex(),
        "dst": (bytes.fromhex("fe80000000000000") + _eui64_iid(dst_le)).hex(),
        "src_port": nhc[1] << 8 | nhc[2], "dst_port": nhc[3] << 8 | nhc[4],
        "checksum": nhc[5] << 8 | nhc[6], "verify": True,
        "cite": f"{rel}:{lines[0]},{lines[1]},{lines[2]} sixlowpan_three_fragments (datagram_size 307, "
                "tag 0x3f), reassembled",
    }]


def pretty_print_example():
    """The frame of the module example of src/wire/pretty_print.rs and the IPv4 line's checksum
    annotation its expected listing shows (format_checksum, src/wire/ip.rs:871-886)."""
    rel = "src/wire/pretty_print.rs"
    text = _read(rel)
    m = re.search(r"let buffer = vec!\[(.*?)\];", text, re.S)
    body = re.sub(r"//[^\n]*", "", m.group(1))
    frame = _parse_array(body)
    lines = re.findall(r"IPv4 src=.*?proto=\w+( \([^)]*\))?\\n", text)
    return [{
        "name": "pretty_print_module_example", "kind": "eth", "bytes": frame.hex(),
        "ipv4_annotation": lines[0] if lines else "",
        "cite": f"{rel}:{text[: m.start()].count(chr(10)) + 1} (module doc example)",
    }]


def icmpv6_check_len():
    """The message-type length rule of Icmpv6Packet::check_len (src/wire/icmpv6.rs), read from the
    source text: the Message enum values, the field ranges, header_len()'s match arms and the list
    of types check_len holds to ``len >= HEADER_END && len >= header_len()``.  Returns the minimum
    length per type value (0 = check_len rejects the type under the default feature set)."""
    rel = "src/wire/icmpv6.rs"
    text = _read(rel)
    enum = re.search(r"pub enum Message\(u8\)\s*\{(.*?)\}", text, re.S).group(1)
    values = {m.group(1): int(m.group(2), 0) for m in re.finditer(r"(\w+)\s*=\s*(0x[0-9a-fA-F]+)", enum)}
    fields = {}
    for m in re.finditer(r"pub const (\w+): (Field|usize) = ([^;]+);", text):
        v = m.group(3).strip()
        if m.group(2) == "Field":
            a, b = v.split("..")
            fields[m.group(1)] = int(eval(b, {}, {}))  # "end" of a literal range such as 8..8 + 16
        else:
            fields[m.group(1)] = int(v, 0)
    hl = re.search(r"pub fn header_len\(&self\) -> usize \{(.*?)\n    \}", text, re.S)
    header_len = {m.group(1): fields[m.group(2)]
                  for m in re.finditer(r"Message::(\w+) => field::(\w+)\.end", hl.group(1))}
    default_len = fields["CHECKSUM"]
    cl = re.search(r"pub fn check_len\(&self\) -> Result<\(\)> \{(.*?)\n    \}", text, re.S)
    arm = re.search(r"match self\.msg_type\(\) \{\s*((?:\|?\s*Message::\w+\s*)+)=>\s*\{\s*if len < field::HEADER_END "
                    r"\|\| len < self\.header_len\(\)", cl.group(1), re.S)
    listed = re.findall(r"Message::(\w+)", arm.group(1))
    line = text[: cl.start()].count("\n") + 1
    table = {}
    for name, val in sorted(values.items(), key=lambda kv: kv[1]):
        if name in listed:
            table[val] = max(fields["HEADER_END"], header_len.get(name, default_len))
        else:
            table[val] = 0  # RplControl: only with feature proto-rpl (not in Cargo.toml's default)
    return {"min_len": {str(k): v for k, v in table.items()}, "names": {str(v): k for k, v in values.items()},
            "generic_min": 4, "cite": f"{rel}:{line} check_len, header_len, mod field; Cargo.toml default features"}


def main():
    kats = []

    def add(name, rel, arr, proto, field, checksum, verify, pre_fill, cite, src=None, dst=None):
        b, line = static_array(rel, arr)
        assert (b[field] << 8 | b[field + 1]) == checksum, (name, hex(checksum))
        kats.append({
            "name": name, "proto": proto, "bytes": b.hex(), "field": field,
            "checksum": checksum, "verify": verify,
            "pre_fill_field": pre_fill,  # field value the reference test had before fill_checksum
            "src": src, "dst": dst,
            "cite": f"{rel}:{line} ({arr}); {cite}",
        })

    add("ipv4_packet", "src/wire/ipv4.rs", "PACKET_BYTES", "ipv4", 10, 0xD56E, True, 0xA5A5,
        "test_deconstruct checksum()==0xd56e & verify (ipv4.rs:745,748); test_construct fills over 0xa5")
    add("ipv4_repr", "src/wire/ipv4.rs", "REPR_PACKET_BYTES", "ipv4", 10, 0xD279, True, 0xA5A5,
        "test_parse with default caps; test_emit over 0xa5 (ipv4.rs:800-803,856-863)")
    add("udp4_packet", "src/wire/udp.rs", "PACKET_BYTES", "udp", 6, 0x124D, True, 0xFFFF,
        "test_deconstruct 0x124d & verify; test_construct set_checksum(0xffff) then fill (udp.rs:398-413)",
        V4_A, V4_B)
    add("udp4_no_checksum", "src/wire/udp.rs", "NO_CHECKSUM_PACKET", "udp", 6, 0x0000, True, None,
        "test_checksum_omitted: parse accepts a zero field (udp.rs:490-500)", V4_A, V4_B)
    add("tcp4_packet", "src/wire/tcp.rs", "PACKET_BYTES", "tcp", 16, 0x01B6, True, 0xEEEE,
        "test_deconstruct 0x01b6 & verify; test_construct set_checksum(0xEEEE) then fill (tcp.rs:1273-1301)",
        V4_A, V4_B)
    add("tcp4_syn", "src/wire/tcp.rs", "SYN_PACKET_BYTES", "tcp", 16, 0x7A8D, True, 0xA5A5,
        "test_parse default caps; test_emit default caps (tcp.rs:1346-1370)", V4_A, V4_B)
    add("icmpv4_echo", "src/wire/icmpv4.rs", "ECHO_PACKET_BYTES", "icmpv4", 2, 0x8EFE, True, 0xA5A5,
        "test_echo_deconstruct 0x8efe & verify; test_echo_construct over 0xa5 (icmpv4.rs:653-669)")
    add("icmpv6_echo", "src/wire/icmpv6.rs", "ECHO_PACKET_BYTES", "icmpv6", 2, 0x19B3, True, 0xA5A5,
        "test_echo_deconstruct 0x19b3 & verify fe80::1->fe80::2; test_echo_construct over 0xa5",
        FE80_1, FE80_2)
    add("icmpv6_pkt_too_big", "src/wire/icmpv6.rs", "PKT_TOO_BIG_BYTES", "icmpv6", 2, 0x0FC9, True,
        0xA5A5, "test_too_big_deconstruct 0x0fc9 & verify; test_too_big_construct over 0xa5",
        FE80_1, FE80_2)
    add("igmp_leave", "src/wire/igmp.rs", "LEAVE_PACKET_BYTES", "igmp", 2, 0x0269, True, 0xA5A5,
        "test_leave_group_deconstruct 0x269 & verify; test_leave_construct over 0xa5")
    add("igmp_report", "src/wire/igmp.rs", "REPORT_PACKET_BYTES", "igmp", 2, 0x08DA, True, 0xA5A5,
        "test_report_deconstruct 0x08da & verify; test_report_construct over 0xa5")
    add("mld_query", "src/wire/mld.rs", "QUERY_PACKET_BYTES", "icmpv6", 2, 0x7374, True, 0xFFFF,
        "test_query_deconstruct 0x7374; test_query_construct fill(ff02::1, ff02::2) over 0xff",
        FF02_1, FF02_2)
    add("mld_report", "src/wire/mld.rs", "REPORT_PACKET_BYTES", "icmpv6", 2, 0x7385, True, 0xFFFF,
        "test_record_deconstruct 0x7385; test_record_construct fill(ff02::1, ff02::2) over 0xff",
        FF02_1, FF02_2)
    add("ndisc_router_advert", "src/wire/ndisc.rs", "ROUTER_ADVERT_BYTES", "icmpv6", 2, 0xA9DE, True,
        0x0000, "test_router_advert_construct fill(fe80::1, fe80::2) over zeros", FE80_1, FE80_2)

    # UDP computed-zero case (udp.rs:427-435): src port 1, dst port 31881, len 8, zero payload,
    # 192.168.1.1 -> .2: fill must write 0xffff.
    kats.append({
        "name": "udp4_zero_checksum", "proto": "udp", "field": 6,
        "bytes": bytes([0, 1, 31881 >> 8, 31881 & 0xFF, 0, 8, 0xFF, 0xFF]).hex(),
        "checksum": 0xFFFF, "verify": True, "pre_fill_field": 0x0000, "src": V4_A, "dst": V4_B,
        "cite": "src/wire/udp.rs:427-435 test_zero_checksum (bytes built from its setters)",
    })

    packets = []
    for b, line in inline_ipv6_packets("src/iface/interface/tests/ipv6.rs"):
        packets.append({"kind": "ip", "bytes": b.hex(), "cite": f"src/iface/interface/tests/ipv6.rs:{line}",
                        "expect": "icmpv6 verified by Icmpv6Repr::parse(default caps) in parse_ipv6"})

    hbh = hop_by_hop_packets("src/iface/interface/tests/ipv6.rs")

    corpus_dir = os.path.join(REF, "fuzz/corpus/packet_parser")
    corpus = []
    for fn in sorted(os.listdir(corpus_dir)):
        with open(os.path.join(corpus_dir, fn), "rb") as f:
            corpus.append({"name": fn, "kind": "eth", "bytes": f.read().hex(),
                           "cite": f"fuzz/corpus/packet_parser/{fn} (0BSD)"})

    nhc = sixlowpan_nhc_udp()
    pretty = pretty_print_example()
    icmp6 = icmpv6_check_len()

    doc = {
        "generator": "tests/golden/make_golden.py",
        "reference": "smoltcp 0.13.1 (/root/reference, Cargo.toml:3)",
        "kat": kats,
        "iface_ipv6_packets": packets,
        "iface_ipv6_hop_by_hop": hbh,
        "fuzz_corpus_frames": corpus,
        "sixlowpan_nhc_udp": nhc,
        "pretty_print": pretty,
        "icmpv6_check_len": icmp6,
    }
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"wrote {OUT}: {len(kats)} KATs, {len(packets)} iface IPv6 packets, {len(corpus)} frames, "
          f"{len(nhc)} 6LoWPAN NHC UDP packets, {len(hbh)} Hop-by-Hop packets")


if __name__ == "__main__":
    main()
