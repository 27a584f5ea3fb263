"""CPU restatement of abft (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

Restates the consensus caller of the vector-clock index, event by event, as the
reference runs it:

* ``Election``        -- abft/election/election.go:11-124,
                         election_math.go:13-114, sort_roots.go:10-25
* ``Store``           -- abft/store.go, store_roots.go:13-93,
                         store_epoch_state.go, store_last_decided_state.go,
                         store_event_confirmed.go, apply_genesis.go:35-44
* ``Orderer``         -- abft/orderer.go, event_processing.go:15-189,
                         frame_decide.go:11-58, bootstrap.go:30-71
* ``Lachesis``        -- abft/lachesis.go:40-104, traversal.go:13-37
* ``IndexedLachesis`` -- abft/indexed_lachesis.go:53-99

The DAG index is any object with the vecfc.Index surface used by abft
(``reset``, ``add``, ``flush``, ``drop_not_flushed``, ``forkless_cause``,
``get_merged_highest_before``): ``vecfc_oracle.Index`` for small DAGs, or
``DenseOracleIndex`` below (the C restatement, keyed by event id) for large ones.

Root order.  ``GetFrameRoots`` returns roots from an LRU cache (append order) or
from the kvdb table in key order (store_roots.go:13-93).  The order changes how
early ``forklessCausedByQuorumOn`` stops and the order votes are summed, never a
result (quorum tests and weighted sums are order-free; ``observedRootsMap``
keeps at most one root per validator because FC(a, r1) and FC(a, r2) for two
fork roots r1, r2 of one validator cannot both hold -- a sees their common
fork and vecfc/forkless_cause.go:49-54 answers false).  Roots are therefore
kept in insertion order.  Event IDs are the tdag event ids (names or creation
indices) instead of sha256 hashes; only identity is used.
"""

from .pos import Validators, WeightCounter

FIRST_FRAME = 1      # bootstrap.go:12-15
FIRST_EPOCH = 1


class ElectionError(RuntimeError):
    pass


class WrongFrameError(RuntimeError):
    """ErrWrongFrame (event_processing.go:11-13)."""


class RootAndSlot(tuple):
    """election.RootAndSlot {ID, Slot{Frame, Validator}} (election.go:35-45)."""

    def __new__(cls, eid, frame, validator):
        return super().__new__(cls, (eid, frame, validator))

    id = property(lambda s: s[0])
    frame = property(lambda s: s[1])
    validator = property(lambda s: s[2])


class Vote:
    __slots__ = ("decided", "yes", "observed_root")

    def __init__(self, decided=False, yes=False, observed_root=None):
        self.decided, self.yes, self.observed_root = decided, yes, observed_root


# ----------------------------------------------------------------------------
# abft/election

class Election:
    def __init__(self, validators, frame_to_decide, observe, get_frame_roots):
        self.observe = observe                       # election.go:72-85
        self.get_frame_roots = get_frame_roots
        self.reset(validators, frame_to_decide)

    def reset(self, validators, frame_to_decide):    # election.go:87-93
        self.validators = validators
        self.frame_to_decide = frame_to_decide
        self.votes = {}
        self.decided_roots = {}

    def _not_decided_roots(self):                    # election.go:95-108
        out = [v for v in self.validators.ids if v not in self.decided_roots]
        if len(out) + len(self.decided_roots) != len(self.validators):
            raise ElectionError("Mismatch of roots")
        return out

    def _observed_roots(self, root, frame):          # election.go:110-121
        return [r for r in self.get_frame_roots(frame) if self.observe(root, r.id)]

    def _observed_roots_map(self, root, frame):      # election.go:123-124 (+ file end)
        m = {}
        for r in self.get_frame_roots(frame):
            if self.observe(root, r.id):
                m[r.validator] = r
        return m

    def process_root(self, new_root):                # election_math.go:13-114
        res = self.choose_atropos()
        if res is not None:
            return res
        if new_root.frame <= self.frame_to_decide:
            return None
        rnd = new_root.frame - self.frame_to_decide
        not_decided = self._not_decided_roots()
        if rnd == 1:
            observed_map = self._observed_roots_map(new_root.id, new_root.frame - 1)
        else:
            observed = self._observed_roots(new_root.id, new_root.frame - 1)
        for subject in not_decided:
            vote = Vote()
            if rnd == 1:
                r = observed_map.get(subject)
                vote.yes = r is not None
                vote.decided = False
                if r is not None:
                    vote.observed_root = r.id
            else:
                yes_v = WeightCounter(self.validators)
                no_v = WeightCounter(self.validators)
                all_v = WeightCounter(self.validators)
                subject_hash = None
                for r in observed:
                    old = self.votes.get((r, subject))
                    if old is None:
                        raise ElectionError("every root must vote for every not decided subject. "
                                            "possibly roots are processed out of order")
                    if old.yes and subject_hash is not None and subject_hash != old.observed_root:
                        raise ElectionError("forkless caused by 2 fork roots => more than 1/3W are Byzantine")
                    vi = self.validators.idxs[r.validator]
                    if old.yes:
                        subject_hash = old.observed_root
                        yes_v.count_by_idx(vi)
                    else:
                        no_v.count_by_idx(vi)
                    if not all_v.count_by_idx(vi):
                        raise ElectionError("forkless caused by 2 fork roots => more than 1/3W are Byzantine")
                if not all_v.has_quorum():
                    raise ElectionError("root must be forkless caused by at least 2/3W of prev roots. "
                                        "possibly roots are processed out of order")
                vote.yes = yes_v.sum >= no_v.sum
                if vote.yes and subject_hash is not None:
                    vote.observed_root = subject_hash
                vote.decided = yes_v.has_quorum() or no_v.has_quorum()
                if vote.decided:
                    self.decided_roots[subject] = vote
            self.votes[(new_root, subject)] = vote
        return self.choose_atropos()

    def choose_atropos(self):                        # sort_roots.go:10-25
        for v in self.validators.ids:                # SortedIDs = idx order
            vote = self.decided_roots.get(v)
            if vote is None:
                return None
            if vote.yes:
                return (self.frame_to_decide, vote.observed_root)
        raise ElectionError("all the roots are decided as 'no', which is possible only "
                            "if more than 1/3W are Byzantine")


# ----------------------------------------------------------------------------
# abft/store*.go (memory store)

class Store:
    def __init__(self):
        self.epoch_state = None          # (epoch, validators)
        self.last_decided_frame = None
        self._open_epoch_db()

    def _open_epoch_db(self):            # store.go:120-127 (fresh epoch tables)
        self.roots = {}                  # frame -> [RootAndSlot]
        self.confirmed = {}              # event id -> frame

    def apply_genesis(self, epoch, validators):          # apply_genesis.go:17-44
        if len(validators) == 0:
            raise ValueError("genesis validators shouldn't be empty")
        if self.last_decided_frame is not None:
            raise ValueError("genesis already applied")
        self._apply_genesis(epoch, validators)

    def _apply_genesis(self, epoch, validators):
        self.epoch_state = (epoch, validators)
        self.last_decided_frame = FIRST_FRAME - 1

    def get_epoch(self):
        return self.epoch_state[0]

    def get_validators(self):
        return self.epoch_state[1]

    def add_root(self, self_parent_frame, root):         # store_roots.go:22-27
        for f in range(self_parent_frame + 1, root.frame + 1):
            self.roots.setdefault(f, []).append(RootAndSlot(root.id, f, root.creator))

    def get_frame_roots(self, f):                        # store_roots.go:52-93
        return self.roots.get(f, [])


# ----------------------------------------------------------------------------
# abft/orderer.go + event_processing.go + frame_decide.go + bootstrap.go

class Orderer:
    def __init__(self, store, get_event, dag_index, crit=None):
        self.store = store
        self.get_event = get_event
        self.dag_index = dag_index
        self.crit = crit or self._panic
        self.election = None
        self.apply_atropos_cb = None
        self.epoch_db_loaded_cb = None

    @staticmethod
    def _panic(err):
        raise err

    # bootstrap.go:30-52
    def bootstrap_orderer(self, apply_atropos=None, epoch_db_loaded=None):
        if self.election is not None:
            raise RuntimeError("already bootstrapped")
        self.apply_atropos_cb = apply_atropos
        self.epoch_db_loaded_cb = epoch_db_loaded
        if self.epoch_db_loaded_cb is not None:
            self.epoch_db_loaded_cb(self.store.get_epoch())
        self.election = Election(self.store.get_validators(), self.store.last_decided_frame + 1,
                                 self.dag_index.forkless_cause, self.store.get_frame_roots)
        self._bootstrap_election()

    # bootstrap.go:54-65
    def reset(self, epoch, validators):
        self.store._apply_genesis(epoch, validators)
        self._reset_epoch_store(epoch)
        self.election.reset(validators, FIRST_FRAME)

    # event_processing.go:15-30
    def build(self, e):
        e.frame = self._calc_frame_idx(e, False)[1]

    # event_processing.go:32-48
    def process(self, e):
        err, sp_frame = self._check_and_save_event(e)
        if err is not None:
            return err
        try:
            self._handle_election(sp_frame, e)
        except ElectionError as ex:
            self.crit(ex)
            return ex
        return None

    def _check_and_save_event(self, e):          # event_processing.go:50-62
        sp_frame, frame = self._calc_frame_idx(e, True)
        if e.frame != frame:
            return WrongFrameError("claimed frame mismatched with calculated"), 0
        if sp_frame != frame:
            self.store.add_root(sp_frame, e)
        return None, sp_frame

    def _handle_election(self, sp_frame, root):  # event_processing.go:64-100
        for f in range(sp_frame + 1, root.frame + 1):
            decided = self.election.process_root(RootAndSlot(root.id, f, root.creator))
            if decided is None:
                continue
            if self._on_frame_decided(*decided):
                break
            if self._bootstrap_election():
                break

    def _bootstrap_election(self):               # event_processing.go:102-122
        while True:
            decided = self._process_known_roots()
            if decided is None:
                break
            if self._on_frame_decided(*decided):
                return True
        return False

    def _process_known_roots(self):              # event_processing.go:124-146
        f = self.store.last_decided_frame + 1
        while True:
            frame_roots = self.store.get_frame_roots(f)
            for it in frame_roots:
                decided = self.election.process_root(it)
                if decided is not None:
                    return decided
            if not frame_roots:
                break
            f += 1
        return None

    def _forkless_caused_by_quorum_on(self, e, f):   # event_processing.go:148-161
        counter = WeightCounter(self.store.get_validators())
        idxs = self.store.get_validators().idxs
        for it in self.store.get_frame_roots(f):
            if self.dag_index.forkless_cause(e.id, it.id):
                counter.count_by_idx(idxs[it.validator])
            if counter.has_quorum():
                break
        return counter.has_quorum()

    def _calc_frame_idx(self, e, check_only):     # event_processing.go:163-189
        sp_frame = 0
        sp = self_parent(e)
        if sp is not None:
            sp_frame = self.get_event(sp).frame
        max_frame = e.frame if check_only else sp_frame + 100
        f = sp_frame
        while f < max_frame and self._forkless_caused_by_quorum_on(e, f):
            f += 1
        if f == 0:
            f = 1
        return sp_frame, f

    # frame_decide.go:11-35
    def _on_frame_decided(self, frame, atropos):
        new_validators = None
        if self.apply_atropos_cb is not None:
            new_validators = self.apply_atropos_cb(frame, atropos)
        if new_validators is not None:
            self.store.last_decided_frame = FIRST_FRAME - 1
            self._seal_epoch(new_validators)
            self.election.reset(new_validators, FIRST_FRAME)
        else:
            self.store.last_decided_frame = frame
            self.election.reset(self.store.get_validators(), frame + 1)
        return new_validators is not None

    def _reset_epoch_store(self, epoch):          # frame_decide.go:37-50
        self.store._open_epoch_db()
        if self.epoch_db_loaded_cb is not None:
            self.epoch_db_loaded_cb(epoch)

    def _seal_epoch(self, new_validators):        # frame_decide.go:52-58
        epoch = self.store.get_epoch() + 1
        self.store.epoch_state = (epoch, new_validators)
        self._reset_epoch_store(epoch)

    # traversal.go:13-37
    def dfs_subgraph(self, head, filt):
        stack = []
        walk = head
        while walk is not None:
            e = self.get_event(walk)
            if e is None:
                raise RuntimeError("event not found %r" % (walk,))
            if filt(e):
                stack.extend(e.parents)
            walk = stack.pop() if stack else None


def self_parent(e):
    """inter/dag/event.go:87-92."""
    if e.seq <= 1 or not e.parents:
        return None
    return e.parents[0]


# ----------------------------------------------------------------------------
# abft/lachesis.go

class Block:
    """lachesis.Block {Atropos, Cheaters} (lachesis/block.go)."""

    def __init__(self, atropos, cheaters):
        self.atropos = atropos
        self.cheaters = cheaters

    def __eq__(self, o):
        return (self.atropos, self.cheaters) == (o.atropos, o.cheaters)

    def __repr__(self):
        return "Block(%r, cheaters=%r)" % (self.atropos, self.cheaters)


class Lachesis(Orderer):
    """``begin_block(block) -> (apply_event, end_block)`` mirrors
    lachesis.ConsensusCallbacks / BlockCallbacks (lachesis/consensus.go)."""

    def __init__(self, store, get_event, dag_index, crit=None):
        super().__init__(store, get_event, dag_index, crit)
        self.begin_block = None

    def _confirm_events(self, frame, atropos, on_confirmed):   # lachesis.go:40-55
        def filt(e):
            if self.store.confirmed.get(e.id, 0) != 0:
                return False
            self.store.confirmed[e.id] = frame
            if on_confirmed is not None:
                on_confirmed(e)
            return True
        self.dfs_subgraph(atropos, filt)

    def _apply_atropos(self, frame, atropos):                 # lachesis.go:57-86
        clock = self.dag_index.get_merged_highest_before(atropos)
        validators = self.store.get_validators()
        cheaters = [vid for ci, vid in enumerate(validators.ids) if clock.is_fork_detected(ci)]
        if self.begin_block is None:
            return None
        apply_event, end_block = self.begin_block(Block(atropos, cheaters))
        self._confirm_events(frame, atropos, apply_event)
        if end_block is not None:
            return end_block()
        return None

    def bootstrap(self, begin_block=None, epoch_db_loaded=None):   # lachesis.go:88-100
        self.bootstrap_orderer(self._apply_atropos, epoch_db_loaded)
        self.begin_block = begin_block


class IndexedLachesis(Lachesis):
    """abft/indexed_lachesis.go:17-99."""

    def __init__(self, store, get_event, dag_indexer, crit=None):
        super().__init__(store, get_event, dag_indexer, crit)
        self.dag_indexer = dag_indexer
        self._dirty = 0

    def build(self, e):                                       # :53-63
        self._dirty += 1
        real_id, e.id = e.id, ("dirty", self._dirty)          # uniqueDirtyID
        try:
            self.dag_indexer.add(e)
            super().build(e)
        finally:
            self.dag_indexer.drop_not_flushed()
            e.id = real_id

    def process(self, e):                                     # :65-82
        try:
            self.dag_indexer.add(e)
            err = super().process(e)
            if err is not None:
                return err
            self.dag_indexer.flush()
            return None
        finally:
            self.dag_indexer.drop_not_flushed()

    def bootstrap(self, begin_block=None):                    # :84-99
        def loaded(epoch):
            self.dag_indexer.reset(self.store.get_validators(), self.get_event)
        super().bootstrap(begin_block, loaded)


# ----------------------------------------------------------------------------
# C-restatement-backed index keyed by event id (for larger DAGs)

class DenseOracleIndex:
    """vecfc.Index surface over ``corc.OracleIndex`` (oracle/csrc/oracle.c)."""

    def __init__(self):
        self.o = None

    def reset(self, validators, get_event=None):
        from .corc import OracleIndex
        self.validators = validators
        self.o = OracleIndex(validators.weights)
        self.pos = {}
        self.ids = []
        self.n_flushed = 0

    def add(self, e):
        ps = []
        for p in e.parents:
            if p not in self.pos:
                raise RuntimeError("processed out of order, parent not found")
            ps.append(self.pos[p])
        rc = self.o.add(self.validators.idxs[e.creator], e.seq, ps)
        if rc != 0:
            raise RuntimeError("oracle add failed: %d" % rc)
        self.pos[e.id] = len(self.ids)
        self.ids.append(e.id)

    def flush(self):
        self.o.flush()
        self.n_flushed = len(self.ids)

    def drop_not_flushed(self):
        self.o.drop_not_flushed()
        for eid in self.ids[self.n_flushed:]:
            del self.pos[eid]
        del self.ids[self.n_flushed:]

    def forkless_cause(self, a, b):
        return bool(self.o.forkless_cause(self.pos[a], self.pos[b]))

    def get_merged_highest_before(self, eid):
        from .vecfc_oracle import HighestBeforeSeq
        return HighestBeforeSeq(raw=self.o.merged_hb(self.pos[eid]))


def new_validators(weights_by_id):
    return Validators(weights_by_id)
