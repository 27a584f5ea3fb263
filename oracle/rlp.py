"""RLP encoding restated from the published go-ethereum `rlp` specification
(github.com/ethereum/go-ethereum v1.9.22, pinned in the reference's go.mod:5-15;
the dependency itself is not vendored in /root/reference).

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of the HIP
library's BranchesInfo write-back (table "B", vecengine/store_branches_info.go:
13-22,57-61).  Pinned to the specification's worked examples
(tests/test_writeback_cpu.py), not to reference outputs: no reference test
holds RLP bytes of BranchesInfo, so byte parity of table "B" is
spec-pinned, not reference-pinned.

Rules used (Yellow Paper appendix B / go-ethereum rlp/encode.go):
  uint x     : 0 -> 0x80; x < 0x80 -> one byte x; else 0x80+len, big-endian
               minimal bytes.
  byte string: one byte < 0x80 -> itself; len <= 55 -> 0x80+len || bytes;
               else 0xB7+len(len) || len || bytes.
  list       : payload = concatenated items; len <= 55 -> 0xC0+len || payload;
               else 0xF7+len(len) || len || payload.
  struct     : list of its exported fields in declaration order.
"""


def _be(n):
    out = b""
    while n:
        out = bytes([n & 0xFF]) + out
        n >>= 8
    return out


def enc_uint(x):
    if x == 0:
        return b"\x80"
    if x < 0x80:
        return bytes([x])
    b = _be(x)
    return bytes([0x80 + len(b)]) + b


def enc_bytes(s):
    s = bytes(s)
    if len(s) == 1 and s[0] < 0x80:
        return s
    if len(s) <= 55:
        return bytes([0x80 + len(s)]) + s
    ln = _be(len(s))
    return bytes([0xB7 + len(ln)]) + ln + s


def enc_list(items):
    payload = b"".join(items)
    if len(payload) <= 55:
        return bytes([0xC0 + len(payload)]) + payload
    ln = _be(len(payload))
    return bytes([0xF7 + len(ln)]) + ln + payload


def encode(v):
    """ints -> uint, bytes/str -> string, lists/tuples -> list (recursively)."""
    if isinstance(v, bool):
        return enc_uint(int(v))
    if isinstance(v, int):
        return enc_uint(v)
    if isinstance(v, str):
        return enc_bytes(v.encode())
    if isinstance(v, (bytes, bytearray)):
        return enc_bytes(v)
    return enc_list([encode(x) for x in v])


def encode_branches_info(last_seq, creator_idxs, by_creators):
    """BranchesInfo{BranchIDLastSeq []idx.Event, BranchIDCreatorIdxs
    []idx.Validator, BranchIDByCreators [][]idx.Validator}
    (vecengine/branches_info.go:9-13) as rlp.EncodeToBytes writes it."""
    return encode([list(last_seq), list(creator_idxs), [list(x) for x in by_creators]])
