"""Python model of the device algorithm (test helper, not product code).

The HIP path (lachesis-base_amd/csrc) does NOT run the reference's per-event
DFS or its marker-absorbing CollectFrom.  It computes, per event e and branch c:

  RAW(e)[c]  = max over parents p of RAW(p)[c];  RAW(e)[br(e)] = seq(e)
  MARK(e)[n] = creator n has >=2 branches at Add(e) time and two non-empty
               branches a != b of n overlap:  first(a) <= RAW(e)[b] and
               first(b) <= RAW(e)[a]                    (no propagation needed)
  LA fill    : for e on branch j, c any branch, h0 = RAW(prev_j)[c] (0 if e
               starts branch j), h1 = RAW(e)[c]:
               LA((c, s))[j] = seq(e) for s in (max(h0, first(c)-1), h1]

This module states that model in plain Python so the tests can check, on
fork-heavy DAGs, that it reproduces the oracle's byte rows exactly
(tests/test_device_model.py).  The HIP kernels implement this model.
"""

MAX_INT32 = 0x7FFFFFFF


class DeviceModel:
    def __init__(self, validators):
        self.v = validators
        V = len(validators)
        self.V = V
        self.last_seq = [0] * V
        self.creator_of = list(range(V))
        self.by_creator = [[i] for i in range(V)]
        self.first_seq = [1] * V
        self.branch_rows = [[] for _ in range(V)]   # branch -> event ids by seq order
        self.ev = {}        # id -> dict(branch, seq, b_before, b_after)
        self.raw = {}       # id -> list
        self.mark = {}      # id -> set(creator)
        self.la = {}        # id -> dict(branch -> seq)

    def B(self):
        return len(self.creator_of)

    def add(self, e):
        me = self.v.idxs[e.creator]
        b_before = self.B()
        sp = e.self_parent()
        br = None
        if sp is None:
            if self.last_seq[me] == 0:
                br = me
        else:
            spb = self.ev[sp]["branch"]
            if self.last_seq[spb] + 1 == e.seq:
                br = spb
        if br is None:
            self.last_seq.append(0)
            self.creator_of.append(me)
            br = len(self.creator_of) - 1
            self.by_creator[me].append(br)
            self.first_seq.append(e.seq)
            self.branch_rows.append([])
        self.last_seq[br] = e.seq
        self.branch_rows[br].append(e.id)
        B = self.B()
        raw = [0] * B
        for p in e.parents:
            pr = self.raw[p]
            for c in range(len(pr)):
                if pr[c] > raw[c]:
                    raw[c] = pr[c]
        raw[br] = e.seq
        marks = set()
        if B > self.V:
            for n in range(self.V):
                bl = self.by_creator[n]
                if len(bl) < 2:
                    continue
                hit = False
                for a in bl:
                    for b in bl:
                        if a != b and raw[a] and raw[b] and \
                                self.first_seq[a] <= raw[b] and self.first_seq[b] <= raw[a]:
                            hit = True
                if hit:
                    marks.add(n)
        self.ev[e.id] = dict(branch=br, seq=e.seq, b_before=b_before, b_after=B)
        self.raw[e.id] = raw
        self.mark[e.id] = marks
        self.la[e.id] = {}
        # range fill
        prev = sp if (sp is not None and self.ev[sp]["branch"] == br) else None
        prev_raw = self.raw[prev] if prev is not None else None
        for c in range(B):
            h0 = prev_raw[c] if (prev_raw is not None and c < len(prev_raw)) else 0
            h1 = raw[c]
            lo = max(h0 + 1, self.first_seq[c])
            for s in range(lo, h1 + 1):
                x = self.branch_rows[c][s - self.first_seq[c]]
                assert br not in self.la[x]
                self.la[x][br] = e.seq

    # reference byte layouts ------------------------------------------------
    def hb_bytes(self, eid):
        import struct
        info = self.ev[eid]
        raw = self.raw[eid]
        marks = self.mark[eid]
        vals = []
        for c in range(info["b_after"]):
            if self.creator_of[c] in marks:
                vals.append((0, MAX_INT32))
            elif raw[c]:
                vals.append((raw[c], self.first_seq[c]))
            else:
                vals.append((0, 0))
        n = info["b_before"]
        for c, v in enumerate(vals):
            if v != (0, 0):
                n = max(n, c + 1)
        return b"".join(struct.pack("<II", *vals[c]) for c in range(n))

    def la_bytes(self, eid):
        import struct
        info = self.ev[eid]
        la = self.la[eid]
        n = max([info["b_before"]] + [j + 1 for j in la])
        return b"".join(struct.pack("<I", la.get(j, 0)) for j in range(n))

    def forkless_cause(self, a, b):
        ia, ib = self.ev[a], self.ev[b]
        raw_a = self.raw[a]
        marks_a = self.mark[a]
        bb = ib["branch"]
        if bb < ia["b_after"] and self.creator_of[bb] in marks_a:
            return False
        la_b = self.la[b]
        hit = set()
        for j, s in la_b.items():
            if j < len(raw_a) and j < ia["b_after"] and self.creator_of[j] not in marks_a \
                    and s <= raw_a[j]:
                hit.add(self.creator_of[j])
        w = sum(self.v.weights[c] for c in hit)
        return w >= self.v.quorum()
