"""The oracle (CPU restatement of the reference) against the reference's own
known-answer tests (tests/golden/kat.json, transcribed by make_kat.py)."""
import pytest

from oracle import oracle


def test_forward_bits(kat):
    for c in kat["forward_bits"]:
        r, (a, b), vals, la = oracle.forward_bits(bytes(c["data"]), c["takes"])
        if "error" in c:
            assert r == c["error"], c["src"]
            if "err_a" in c:
                assert a == c["err_a"], c["src"]
            if "err_b" in c:
                assert b == c["err_b"], c["src"]
        else:
            assert r == 0 and vals == c["vals"], c["src"]
        if "len_after" in c:
            assert la == c["len_after"], c["src"]


def test_backward_bits(kat):
    for c in kat["backward_bits"]:
        r, (a, b), vals, lb, la = oracle.backward_bits(bytes(c["data"]), c["takes"])
        if "error" in c:
            assert r == c["error"], c["src"]
            if "err_a" in c:
                assert a == c["err_a"], c["src"]
            if "err_b" in c:
                assert b == c["err_b"], c["src"]
        else:
            assert r == 0, c["src"]
            if "vals" in c:
                assert vals == c["vals"], c["src"]
            if "len_before" in c:
                assert lb == c["len_before"], c["src"]
        if "len_after" in c:
            assert la == c["len_after"], c["src"]


def test_backward_take_zero_after_byte_boundary():
    # tests/parsing.rs:348-358 weird_bug_ok_should_not_panic
    for i in range(15):
        oracle.backward_bits(bytes([0b10100000, 0b01111000]), [i, 0])


def test_parse_fse_table(kat):
    for c in kat["parse_fse_table"]:
        al, dist, bits_left = oracle.parse_fse_table(bytes(c["data"]))
        assert (al, dist, bits_left) == (c["al"], c["dist"], c["bits_left"]), c["src"]


def test_fse_from_distribution(kat):
    for c in kat["fse_from_distribution"]:
        st = oracle.fse_from_distribution(c["al"], c["dist"])
        for k, v in c["states"].items():
            assert list(st[int(k)]) == v, c["src"]
    for c in kat["fse_table_parse"]:
        al, dist, _ = oracle.parse_fse_table(bytes(c["data"]))
        st = oracle.fse_from_distribution(al, dist)
        for k, v in c["states"].items():
            assert list(st[int(k)]) == v, c["src"]


def test_fse_and_alternating_decode(kat):
    for c in kat["fse_decode"]:
        assert oracle.fse_decode(c["table"], c["al"], bytes(c["stream"]), len(c["symbols"])) == c["symbols"], c["src"]
    for c in kat["alternating_decode"]:
        assert oracle.alternating_decode(c["table"], c["al"], bytes(c["stream"]), len(c["symbols"])) == c["symbols"], c["src"]


def test_huffman(kat):
    for c in kat["huffman_weights_decode"]:
        assert oracle.huffman_weights_decode(c["weights"], bytes(c["stream"])) == c["out"].encode(), c["src"]
    for c in kat["huffman_parse_decode"]:
        cons, out = oracle.huffman_parse_decode(bytes(c["desc"]), bytes(c["stream"]))
        assert cons == len(c["desc"]) and out == c["out"].encode(), c["src"]
    for c in kat["huffman_widths"]:
        _, w = oracle.huffman_widths(bytes(c["desc"]))
        for k, v in c["widths_at"].items():
            assert w[int(k)] == v, c["src"]


def test_execute_sequences(kat):
    for c in kat["execute_sequences"]:
        assert oracle.execute_sequences([tuple(s) for s in c["seqs"]], bytes(c["literals"])) == bytes(c["out"]), c["src"]


def test_header(kat):
    for c in kat["header_parse"]:
        if "error" in c:
            with pytest.raises(oracle.OracleError) as ex:
                oracle.header_parse(bytes(c["data"]))
            assert ex.value.code == c["error"], c["src"]
            continue
        h, _ = oracle.header_parse(bytes(c["data"]))
        assert h["content_checksum_flag"] == c["checksum"], c["src"]
        assert h["window_size"] == c["window"], c["src"]
        assert h["content_size"] == c["fcs"], c["src"]
        assert h["dictionnary_id"] == c["dict"], c["src"]
    for c in kat["window_descriptor"]:
        # a non-single-segment header with no FCS exposes the descriptor alone
        h, _ = oracle.header_parse(bytes([0x00, c["byte"]]))
        assert h["window_size"] == c["window"], c["src"]


def expected_frames_output(c):
    if "out_rle" in c:
        b, n, t = c["out_rle"]
        return bytes([b]) * n + bytes([t])
    return bytes(c.get("out", []))


def test_frames(kat):
    for c in kat["frames"]:
        data = bytes(c["data"])
        st, out = oracle.decompress_status(data)
        if c.get("no_panic"):
            assert st != -90, c["src"]
            continue
        if "error" in c:
            assert st == c["error"], (c["src"], st)
            continue
        assert st == 0 and out == expected_frames_output(c), c["src"]
        if "skippable_out" in c:
            st, out = oracle.decompress_status(data, True)
            assert st == 0 and out == bytes(c["skippable_out"]), c["src"]
