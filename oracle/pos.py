"""Validator set restatement (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

Follows ``inter/pos/validators.go`` and ``inter/pos/sort.go``:

* idx order = sort by (weight desc, ID asc)           -- sort.go:16-22
* weights of zero are dropped by the builder           -- validators.go:39-45
* total weight must stay <= MaxUint32/2                -- validators.go:101-110
* quorum = total*2/3 + 1 (uint32 arithmetic)           -- validators.go:187-189
"""

MAX_UINT32 = 0xFFFFFFFF


class Validators:
    def __init__(self, weights_by_id):
        vals = [(vid, w) for vid, w in weights_by_id.items() if w != 0]
        # sort.go:16-22: weight desc, then ID asc
        vals.sort(key=lambda t: (-t[1], t[0]))
        self.ids = [v for v, _ in vals]
        self.weights = [w for _, w in vals]
        self.idxs = {v: i for i, v in enumerate(self.ids)}
        total = 0
        for w in self.weights:
            total += w
            if total > MAX_UINT32:
                raise OverflowError("validators weight overflow")
        if total > MAX_UINT32 // 2:
            raise OverflowError("validators weight overflow")
        self.total_weight = total

    @classmethod
    def equal(cls, ids, weight=1):
        return cls({i: weight for i in ids})

    def __len__(self):
        return len(self.ids)

    def quorum(self):
        # validators.go:187-189 (uint32: total <= MaxUint32/2, so 2*total fits)
        return (self.total_weight * 2 // 3 + 1) & MAX_UINT32


class WeightCounter:
    """inter/pos/stake.go:31-60: per-idx dedupe, sum, quorum test."""

    def __init__(self, validators):
        self.v = validators
        self.already = [False] * len(validators)
        self.quorum = validators.quorum()
        self.sum = 0

    def count_by_idx(self, i):
        if self.already[i]:
            return False
        self.already[i] = True
        self.sum += self.v.weights[i]
        return True

    def has_quorum(self):
        return self.sum >= self.quorum
