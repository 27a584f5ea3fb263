"""CPU checks of the write-back checker: the RLP restatement (oracle/rlp.py) on
the specification's worked examples (go-ethereum rlp v1.9.22 / Yellow Paper
appendix B), and the oracle's flushable tables behave as the reference's
(vecengine/index.go:78-96: Puts are invisible to the store until Flush,
DropNotFlushed discards them)."""

import pytest

from oracle import pos, rlp, tdag
from oracle import vecfc_oracle as vo


@pytest.mark.parametrize("value,encoded", [
    (0, "80"), (15, "0f"), (127, "7f"), (128, "8180"), (256, "820100"), (1024, "820400"),
    (0xFFFFFF, "83ffffff"), (0xFFFFFFFF, "84ffffffff"),
    (b"", "80"), (b"dog", "83646f67"), ([], "c0"), ([b"cat", b"dog"], "c88363617483646f67"),
    ([[], [[]], [[], [[]]]], "c7c0c1c0c3c0c1c0"),
    (b"Lorem ipsum dolor sit amet, consectetur adipisicing elit",
     "b838" + b"Lorem ipsum dolor sit amet, consectetur adipisicing elit".hex()),
    (list(range(1, 57)), "f838" + bytes(range(1, 57)).hex()),
])
def test_rlp_spec_examples(value, encoded):
    assert rlp.encode(value).hex() == encoded


def test_branches_info_rlp_layout():
    """BranchesInfo is a 3-field struct: list(list uint, list uint, list(list uint))."""
    got = rlp.encode_branches_info([3, 0, 2], [0, 1, 0], [[0, 2], [1]])
    assert got.hex() == "ce" + "c3038002" + "c3800180" + "c5c28002c101"
    # long lists switch to the 0xF8 header
    n = 60
    big = rlp.encode_branches_info([200] * n, list(range(n)), [[i] for i in range(n)])
    assert big[0] == 0xF9 and rlp.encode([200] * n)[:2].hex() == "f878"


def test_oracle_tables_flush_and_drop():
    nodes, evs = tdag.rand_fork_dag(6, 12, 3, cheaters=2, forks_count=4, seed=3)
    validators = pos.Validators.equal(nodes)
    store = {e.id: e for e in evs}
    o = vo.Index()
    o.reset(validators, store.get)
    for e in evs[:20]:
        o.add(e)
    assert len(o.tbl_hb.dirty) == 20 and not o.tbl_hb.flushed
    o.flush()
    assert len(o.tbl_hb.flushed) == 20 and not o.tbl_hb.dirty and b"c" in o.tbl_binfo.flushed
    for e in evs[20:30]:
        o.add(e)
    # LowestAfter rows of old events are rewritten by the new events' DFS Visits
    assert set(o.tbl_la.dirty) - {e.id for e in evs[20:30]}
    o.drop_not_flushed()
    assert not o.tbl_la.dirty and o.get_highest_before(evs[25].id) is None
