"""The causal attention backward's work plan (attention_lds.hip make_plan, read through the host-only
rs_attn_bwd_plan; no GPU): every (tile, chunk) pair of every split is covered exactly once, each split tile's
two halves share one LDS slot (writer = lower half, reader = upper half), writers precede whole tiles and
readers in every wave's list, and the slowest wave does less than the round-robin dealing's worst wave and at most
2 chunks over the even share."""
import ctypes as C

import numpy as np
import pytest

PLAN_S, NW, PLAN_I = 4, 8, 6
HANDICAP = 3   # attention_lds.hip LOADER_HANDICAP: plan chunks the loader wave's staging stream is worth


def plan(B, T, H, dkv):
    import rbm_amd._lib as L
    lib = L.lib()
    buf = (C.c_uint32 * (PLAN_S * NW * PLAN_I))()
    ns = C.c_int()
    rc = lib.rs_attn_bwd_plan(B, T, H, int(dkv), buf, C.byref(ns))
    return rc, ns.value, np.frombuffer(buf, dtype=np.uint32).reshape(PLAN_S, NW, PLAN_I)


def chunks(T, dkv):
    """(tile -> [chunk begin, end)) of the pass: dQ tile t scans key chunks [0, ceil((t+1)/2)); dK/dV tile t scans
    query chunks [t // 2, ceil(T / 32))."""
    nq, nqc = -(-T // 16), -(-T // 32)
    return {t: ((t // 2, nqc) if dkv else (0, (t + 2) // 2)) for t in range(nq)}


@pytest.mark.parametrize("dkv", [False, True])
@pytest.mark.parametrize("B,T,H", [(128, 200, 1), (64, 200, 2), (128, 256, 1), (16, 128, 1), (8, 200, 1)])
def test_plan_invariants(B, T, H, dkv):
    rc, ns, p = plan(B, T, H, dkv)
    assert rc == 0, rc
    want = chunks(T, dkv)
    nq = len(want)
    for sp in range(ns):
        tiles = list(range(sp, nq, ns))
        rr = [sum(want[t][1] - want[t][0] for t in tiles[w::NW]) for w in range(NW)]   # round robin, whole tiles
        total = sum(rr)
        covered = {}
        slots = {}
        loads = []
        for w in range(NW):
            roles, load = [], 0
            for it in range(PLAN_I):
                e = int(p[sp, w, it])
                if not e >> 31:
                    assert all(int(x) >> 31 == 0 for x in p[sp, w, it:]), "items must be packed"
                    break
                tile, cb, ce, role, slot = e & 255, (e >> 8) & 255, (e >> 16) & 255, (e >> 24) & 3, (e >> 26) & 15
                assert tile % ns == sp and tile < nq
                for c in range(cb, ce):
                    assert (tile, c) not in covered, "pair covered twice"
                    covered[(tile, c)] = True
                if role:
                    slots.setdefault(slot, []).append((role, tile, cb, ce))
                roles.append(role)
                load += ce - cb
            order = {1: 0, 0: 1, 2: 2}
            assert [order[r] for r in roles] == sorted(order[r] for r in roles), "writers, wholes, readers"
            loads.append(load)
        expect = {(t, c) for t in range(sp, nq, ns) for c in range(*want[t])}
        assert set(covered) == expect
        for slot, items in slots.items():
            assert sorted(r for r, *_ in items) == [1, 2], (slot, items)
            (_, t1, b1, e1), (_, t2, b2, e2) = sorted(items)
            assert t1 == t2 and (e2 == b1 or e1 == b2)            # two halves of one tile
            writer = [it for it in items if it[0] == 1][0]
            assert writer[2] == min(b1, b2)                        # the writer holds the lower half
        loads[NW - 1] += HANDICAP                            # the loader wave streams the operand images first
        assert max(loads) < max(rr) + HANDICAP               # better than round robin's slowest wave
        assert max(loads) <= -(-(total + HANDICAP) // NW) + 2   # near the even share


def test_plan_falls_back_for_short_sequences():
    rc, _, _ = plan(128, 50, 1, False)
    assert rc != 0
