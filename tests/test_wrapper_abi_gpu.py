"""The single-object call sequences of the C# plug points, through the C ABI.

`GpuPNCounter` / `GpuORSet` below are line-for-line Python stand-ins of the C# classes a maintainer adds
(`GpuPNCounter : CRDT`, `GpuORSet : CRDT`, MergeSharp/MergeSharp/CRDTBase.cs:40-80, wrapped by
`GpuPNCounterWrapper` / `GpuORSetWrapper : ISafeCRDTWrapper`, BFT-CRDT/SafeCRDTs/SafeCRDT.cs:10-17, and
registered in SafeCRDTManager.TypeMap, SafeCRDTManager.cs:20-23): each object is one row / set of a shared
device store, and every method is the exact ABI sequence of its C# counterpart —
  ctor                                  jg_pnc_intern (own replica = column 0) / a fresh set id
  Update(1|2, args) / Add / Remove / Clear   jg_pnc_apply_ops / jg_orset_names_sync + jg_orset_apply_ops
  GetLastSynchronizedUpdate().Encode()  jg_pnc_encode_json / jg_orset_read_sets (+ the host JSON writer)
  DecodePropagationMessage(bytes)       no call (the bytes are kept; the device decodes them)
  ApplySynchronizedUpdate(msg)          jg_pnc_merge_json / jg_orset_merge_json (+ jg_orset_wave_names)
  Query / LookupAll / Contains          jg_pnc_values / jg_orset_lookup_all / jg_orset_contains
The scenarios are the reference's (PNCounterTests.cs, ORSetTests.cs) with their literal expected
values; messages travel as bytes between objects exactly as SafeCRDT.ApplyUpdateStable
(SafeCRDT.cs:80-83) and ReplicationManager.ReceivedUpdateSyncMsg (ReplicationManager.cs:327-344) pass
them, and PN-Counter bytes are checked against the oracle's System.Text.Json restatement.
"""
import numpy as np
import pytest

import janus_gpu as jg
import jsongen as J
import oracle_ref as orc

pytestmark = pytest.mark.gpu

_rng = np.random.default_rng(0xC5)


def _guid():
    lo, hi = (int(x) for x in _rng.integers(1, 1 << 63, 2, dtype=np.uint64))
    return lo, hi


class GpuStores:
    """The process-wide device stores the C# GpuStores singleton owns (one context per device)."""

    def __init__(self, ctx):
        self.pnc = jg.PNCStore(ctx, 256, 8, 4)  # the reference's int width
        self.orset = jg.ORSetStore(ctx)
        self.next_row = self.next_set = 0

    def close(self):
        self.pnc.close()
        self.orset.close()


class StateMsg:
    """GpuStateMsg : PropagationMessage — the encoded state; Encode() returns it, Decode(bytes) keeps it."""

    def __init__(self, data: bytes):
        self.data = data

    def Encode(self) -> bytes:
        return self.data


class GpuPNCounter:
    def __init__(self, st: GpuStores):
        self.st, self.row = st, st.next_row
        st.next_row += 1
        self.replica = _guid()  # PNCounter(): replicaIdx = Guid.NewGuid(), P = N = {self: 0} (PNCounters.cs:73-81)
        assert int(st.pnc.intern([self.row], [self.replica[0]], [self.replica[1]])[0]) == 0

    def Increment(self, i: int):  # PNCounters.cs:97-101
        self.st.pnc.apply_ops([self.row], [0], [i], [0])

    def Decrement(self, i: int):  # PNCounters.cs:108-112
        self.st.pnc.apply_ops([self.row], [0], [i], [1])

    def Get(self) -> int:  # PNCounters.cs:87-90
        v, ovf = self.st.pnc.values([self.row])
        if ovf[0]:
            raise OverflowError("Arithmetic operation resulted in an overflow.")
        return int(v[0])

    def GetLastSynchronizedUpdate(self) -> StateMsg:
        return StateMsg(self.st.pnc.encode_json([self.row])[0])

    def DecodePropagationMessage(self, data: bytes) -> StateMsg:
        return StateMsg(data)

    def ApplySynchronizedUpdate(self, m: StateMsg):
        self.st.pnc.merge_json([self.row], [m.Encode()])


class GpuPNCounterWrapper:
    """PNCounterWrapper (BFT-CRDT/SafeCRDTs/PNCounterWrapper.cs:28-47) over GpuPNCounter."""

    def __init__(self, crdt: GpuPNCounter):
        self.crdt = crdt

    def Query(self, args=None):
        return self.crdt.Get()

    def Update(self, op: int, args):
        arg = int(args[0])  # (int)args[0] before the switch
        if op == 1:
            self.crdt.Increment(arg)
        elif op == 2:
            self.crdt.Decrement(arg)
        else:
            raise ValueError("Invalid PNC method name")  # InvalidOperationException
        return True


class GpuORSet:
    """ORSet<string?> (ORSet.cs:78-327) as one set of the device store, with its element interning."""

    def __init__(self, st: GpuStores):
        self.st, self.set = st, st.next_set
        st.next_set += 1
        self.ids, self.names = {}, []  # live element -> id (first insertion; reset by Clear), id -> element

    def _id(self, e, create):
        if e is None:
            return jg.NULL_ELEM
        if e in self.ids:
            return self.ids[e]
        if not create:
            return jg.NULL_ELEM - 1  # never issued: no record carries it (Contains is false, ORSet.cs:170-173)
        self.ids[e] = len(self.names)
        self.names.append(e)
        self.st.orset.names_sync(sets=[self.set], next_ids=[len(self.names)], cleared=[0],
                                 names=[(self.set, self.ids[e], e.encode())])
        return self.ids[e]

    def _op(self, op, e, tag=(0, 0)):
        return bool(self.st.orset.apply_ops([self.set], [self._id(e, op == 1)], [op], [tag[0]], [tag[1]])[0])

    def Add(self, e):  # ORSet.cs:134-153, Guid.NewGuid()
        return self._op(1, e, _guid())

    def Remove(self, e):  # ORSet.cs:161-186
        return self._op(2, e)

    def Clear(self):  # ORSet.cs:192-198: later adds take new ids
        self._op(3, None)
        self.ids = {}
        self.st.orset.names_sync(sets=[self.set], next_ids=[len(self.names)], cleared=[1])

    def LookupAll(self):  # ORSet.cs:204-227
        ids = self.st.orset.lookup_all([self.set])[0]
        return [None if int(i) == jg.NULL_ELEM else self.names[int(i)] for i in ids]

    def Contains(self, e):
        return bool(self.st.orset.contains([self.set], [self._id(e, False)])[0])

    def GetLastSynchronizedUpdate(self) -> StateMsg:
        (add, rem), = self.st.orset.read_sets([self.set])
        view = lambda recs, r: orc.enum_view(recs, r)  # noqa: E731  (the host writer's order: jg_tagrec.ord)

        def dmap(recs, r):
            out, nulls = [], []
            for key, lo, hi in view(recs, r):
                e = int(key) & 0xFFFFFFFF
                if e == jg.NULL_ELEM:
                    nulls.append((int(lo), int(hi)))
                elif out and out[-1][0] == self.names[e]:
                    out[-1][1].append((int(lo), int(hi)))
                else:
                    out.append((self.names[e], [(int(lo), int(hi))]))
            return out, nulls

        a, na = dmap(add, False)
        r, nr = dmap(rem, True)
        return StateMsg(J.encode_orset(a, r, na, nr))

    def DecodePropagationMessage(self, data: bytes) -> StateMsg:
        return StateMsg(data)

    def ApplySynchronizedUpdate(self, m: StateMsg):
        self.st.orset.merge_json([self.set], [m.Encode()])
        for s, i, name in self.st.orset.wave_names():  # ids the merge issued, in first-insertion order
            assert s == self.set and i == len(self.names)
            self.names.append(name.decode())
            self.ids[name.decode()] = i


@pytest.fixture
def st(ctx):
    s = GpuStores(ctx)
    yield s
    s.close()


def _merge(dst, src):  # dst.ApplySynchronizedUpdate(dst.DecodePropagationMessage(src.GetLastSynchronizedUpdate().Encode()))
    dst.ApplySynchronizedUpdate(dst.DecodePropagationMessage(src.GetLastSynchronizedUpdate().Encode()))


def test_pncounter_scenarios(st):
    # PNCounterTests.cs:8-19 through the wrapper's op ids (the command layer's path)
    w = GpuPNCounterWrapper(GpuPNCounter(st))
    for op, v in ((1, 5), (2, 8), (1, 10), (2, 3)):
        assert w.Update(op, [v]) is True
    assert w.Query() == 4
    with pytest.raises(ValueError):
        w.Update(3, [1])
    # PNCounterTests.cs:21-38 and :46-66
    p1, p2 = GpuPNCounter(st), GpuPNCounter(st)
    p1.Increment(5); p1.Decrement(1)
    p2.Increment(2); p1.Decrement(2)
    _merge(p1, p2)
    assert p1.Get() == 5 - 1 + 2 - 2
    # the bytes are the reference's: {"pVector":{self:.., other:..},"nVector":{..}} in insertion order
    got = p1.GetLastSynchronizedUpdate().Encode()
    exp = orc.json_encode_pnc([p1.replica[0], p2.replica[0]], [p1.replica[1], p2.replica[1]], [5, 2], [3, 0], 4)
    assert got == exp
    # checked Sum: PNCounters.cs:89
    a, b = GpuPNCounter(st), GpuPNCounter(st)
    a.Increment(2**31 - 1)
    b.Increment(1)
    _merge(a, b)
    with pytest.raises(OverflowError):
        a.Get()


def test_orset_scenarios(st):
    # ORSetTests.cs:102-129 (Multiple; order-sensitive at :113)
    s1, s2 = GpuORSet(st), GpuORSet(st)
    s1.Add("1"); s2.Add("2")
    _merge(s1, s2)
    assert s1.LookupAll() == ["1", "2"] and len(s1.LookupAll()) == 2
    assert s2.LookupAll() == ["2"]
    _merge(s2, s1)
    assert sorted(s1.LookupAll()) == sorted(s2.LookupAll())
    s1.Remove("2")
    assert s1.LookupAll() == ["1"]
    s1.Add("2"); s2.Remove("2")
    _merge(s1, s2)
    assert sorted(s1.LookupAll()) == ["1", "2"]
    # ORSetTests.cs:314-347 (MergeNull, MergeNull2; order-sensitive at :327, :343, :346)
    a, b = GpuORSet(st), GpuORSet(st)
    a.Add("hi"); a.Add(None)
    assert not b.Remove(None)
    _merge(a, b)
    assert a.LookupAll() == ["hi", None]
    c, d = GpuORSet(st), GpuORSet(st)
    c.Add("hi"); c.Add(None)
    d.Add(None); d.Remove(None)
    _merge(d, c)
    assert d.LookupAll() == ["hi", None]
    _merge(c, d)
    assert c.LookupAll() == ["hi", None]
    # ORSetTests.cs:453-474 (EncodeDecode; order-sensitive at :473) and SingleORSetValueType1 :10-40
    e1, e2 = GpuORSet(st), GpuORSet(st)
    e1.Add("a"); e1.Add("b")
    e2.Add("a"); e2.Add("b"); e2.Remove("b")
    _merge(e1, e2)
    assert e1.LookupAll() == ["a", "b"]
    f = GpuORSet(st)
    f.Add("1"); f.Add("2")
    assert f.Remove("1") and not f.Remove("3")
    f.Add("3")
    assert sorted(f.LookupAll()) == ["2", "3"]
    f.Clear()
    assert f.LookupAll() == [] and not f.Contains("1")
    f.Add("1")
    assert f.Contains("1") and f.LookupAll() == ["1"]


def test_orset_bytes_round_trip_and_enumeration(st):
    """GetLastSynchronizedUpdate().Encode() of a merged set decodes (oracle Decode) to the same Dictionaries
    and HashSets, in the same enumeration order, that the oracle's Merge built."""
    s, r = GpuORSet(st), GpuORSet(st)
    for e in ("b", "a", "b", None, None):
        s.Add(e)
    assert s.Remove("b") and s.Remove("a")
    r.Add("a"); r.Add("b")
    _merge(r, s)
    dec = orc.json_decode_orset(r.GetLastSynchronizedUpdate().Encode())
    assert dec is not None
    adds = [(name.decode(), len(tags)) for side, is_null, name, tags in dec if side == 0 and not is_null]
    rems = [name.decode() for side, is_null, name, tags in dec if side == 1 and not is_null]
    assert adds == [("a", 2), ("b", 3)]  # r's own tag first, then s's in s's order
    assert rems == ["b", "a"]            # the tombstone Dictionary in first-insertion order (s's Removes)
