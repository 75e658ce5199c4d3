"""Host model of the GPU nearest-neighbour chain's launch protocol
(drep_amd/csrc/linkage.hip, k_nn_step) -- a design tool, not product code.

The GPU chain makes scipy's nn_chain decisions (drep/d_cluster.py:447-453 ->
scipy.cluster.hierarchy.linkage) at the START of each launch from the row
minima ("partials") the previous launch reduced: P1 = the chain top's row,
P2 = the merged row or a speculated merged row, P3 = a speculated row of the
element below.  This script replays that protocol on the host with numpy on a
dense n x n float64 matrix, so a change of protocol can be judged by two
numbers before any kernel is written: the launch count, and whether Z is
still bit-identical to scipy's.

  python tools/chain_sim.py <common.npy> [--policy r4|r5] [--n N]

<common.npy>: the condensed shared-hash counts (uint16, s = 1000, every sketch
full) of the configs workload, e.g. from oracle.sketch_synth + oracle.allpairs.
"""
import argparse
import sys
import time

import numpy as np

INF = np.inf


class Sim:
    def __init__(self, D, policy="r4", method="average"):
        self.method = method
        self.D = D
        self.n = n = D.shape[0]
        self.size = np.ones(n, dtype=np.int64)
        self.chain = [0]
        self.Z = []
        self.policy = policy
        self.stats = dict(launches=0, twice=0, scans=0, specwin=0, m0=0, merges=0, w_merge=0, w_recip=0,
                          known_merges=0, known_spec=0,
                          rows_known_at_start=0, rows_known_after_partials=0, rows_known_after_decision=0)

    # ---- row minima (smallest index among equal minima, as the GPU's argmin)
    def rowmin(self, vals, mask):
        v = np.where(mask, vals, INF)
        i = int(np.argmin(v))
        return (float(v[i]), i) if v[i] < INF else (INF, -1)

    def active(self):
        return self.size > 0

    def lw(self, dx, dy, nx, ny):       # scipy's Lance-Williams updates and rounding
        if self.method == "complete":
            return np.maximum(dx, dy)
        if self.method == "weighted":
            return 0.5 * (dx + dy)
        return (nx * dx + ny * dy) / float(nx + ny)

    def apply_merge(self, a, b):
        """scipy: x = a < y = b; new row/column b, size[a] = 0"""
        D, size = self.D, self.size
        na, nb = size[a], size[b]
        act = self.active().copy()
        act[a] = act[b] = False
        u = self.lw(D[a], D[b], float(na), float(nb))
        D[b, act] = u[act]
        D[act, b] = u[act]
        size[a] = 0
        size[b] = na + nb

    def p1(self, t):
        m = self.active().copy()
        m[t] = False
        return self.rowmin(self.D[t], m)

    def spec_rows(self, t, sb, w):
        """the row U = LW(D[t], D[sb]) would form (index max(t, sb)) and w's row
        after that merge: their minima (P2, P3)"""
        D, size = self.D, self.size
        x, y = min(t, sb), max(t, sb)
        m = self.active().copy()
        m[t] = m[sb] = False
        U = self.lw(D[x], D[y], float(size[x]), float(size[y]))
        p2 = self.rowmin(U, m)
        mw = m.copy()
        mw[w] = False
        vw = np.where(mw, D[w], INF)
        iw = int(np.argmin(vw))
        best = (float(vw[iw]), iw) if vw[iw] < INF else (INF, 1 << 30)
        cand = (float(U[w]), y)
        if cand[0] < best[0] or (cand[0] == best[0] and cand[1] < best[1]):
            best = cand
        return p2, best

    def run(self):
        n, D, st = self.n, self.D, self.stats
        chain = self.chain
        decide = False
        P1 = P2 = P3 = None
        mrow = -1
        spec = 0
        k = 0
        known = None
        P2y = None
        while k < n - 1:
            st["launches"] += 1
            pend = None
            prev_known, known = known, None
            # rows a launch could start loading before its decision: those the
            # state names (top, below and the two under them), and those the
            # previous launch's partials name (their argmins)
            cand0 = set(chain[-4:])
            cand1 = cand0 | {r[1] for r in (P1, P2, P3) if r is not None and r[1] >= 0}
            # ---- decisions at the start of the launch
            if decide and prev_known:
                # the previous launch knew this launch's first decision (a merge of
                # the top with the element below) and speculated on it: no P1 needed
                top, below = chain[-1], chain[-2]
                a, b = min(top, below), max(top, below)
                self.Z.append((a, b, D[top, below], self.size[a] + self.size[b]))
                pend = (a, b)
                k += 1
                chain.pop(); chain.pop()
                st["known_merges"] += 1
                if not chain and k < n - 1:
                    act = self.active()
                    chain.append(next(i for i in range(n) if i == b or (i != a and act[i])))
                elif chain and k < n - 1:
                    r3 = P3
                    L = len(chain)
                    dp2 = D[chain[-1], chain[-2]] if L > 1 else INF
                    wpush = r3[1] >= 0 and not (L > 1 and not (r3[0] < dp2))
                    bpush = r3[1] == b and P2[1] >= 0 and P2[0] < r3[0]
                    if wpush and (r3[1] != b or bpush):
                        chain.append(r3[1])
                        st["specwin"] += 1
                        if bpush:
                            chain.append(P2[1])
                    elif r3[1] >= 0 and not wpush:
                        st["w_merge"] += 1
                        known = "wmerge"
                    elif wpush and r3[1] == b:
                        st["w_recip"] += 1
                        chain.append(b)
                        known = "recip"
            elif decide:
                r = P1
                for d in range(2):
                    top = chain[-1]
                    below = chain[-2] if len(chain) > 1 else -1
                    dp = D[top, below] if below >= 0 else INF
                    if len(chain) > 1 and not (r[0] < dp):
                        a, b = min(top, below), max(top, below)
                        self.Z.append((a, b, dp, self.size[a] + self.size[b]))
                        pend = (a, b)
                        k += 1
                        chain.pop(); chain.pop()
                        if not chain and k < n - 1:
                            act = self.active()
                            f = next(i for i in range(n) if i == b or (i != a and act[i]))
                            chain.append(f)
                        elif d == 0 and spec and chain and k < n - 1:
                            r3 = P3
                            L = len(chain)
                            dp2 = D[chain[-1], chain[-2]] if L > 1 else INF
                            wpush = r3[1] >= 0 and not (L > 1 and not (r3[0] < dp2))
                            bpush = r3[1] == b and P2[1] >= 0 and P2[0] < r3[0]
                            if wpush and (r3[1] != b or bpush):
                                chain.append(r3[1])
                                st["specwin"] += 1
                                if bpush:
                                    chain.append(P2[1])
                            elif r3[1] >= 0 and not wpush:
                                st["w_merge"] += 1          # w's decision: merge with the element below it
                                if self.policy in ("r5", "r5c"):
                                    known = "wmerge"
                            elif wpush and r3[1] == b:
                                st["w_recip"] += 1          # w pushes b, b merges back with w
                                if self.policy in ("r5", "r5c"):
                                    chain.append(b)
                                    known = "recip"
                        break
                    chain.append(r[1])
                    if r[1] != mrow or mrow < 0 or d == 1:
                        break
                    r = P2y if P2y is not None else P2
                    st["twice"] += 1
            decide = True
            if k >= n - 1:
                break
            # ---- the launch's work: apply the merge, reduce the rows
            if pend:
                self.apply_merge(*pend)
                st["merges"] += 1
            else:
                st["scans"] += 1
            mrow = pend[1] if pend else -1
            t = chain[-1]
            L = len(chain)
            P1 = self.p1(t)
            spec = 0
            need = set(pend) if pend else set()
            if known:
                need |= set(chain[-3:])
            else:
                need.add(t)
                if L >= 3 and (not pend or (chain[-2] == pend[1] and t != pend[1])):
                    need |= set(chain[-3:])
            need.discard(pend[1] if pend else -1)   # (the merged row is computed, not loaded, where it is spec'd)
            if pend:
                need.add(pend[0]); need.add(pend[1])
            if need <= cand0:
                st["rows_known_at_start"] += 1
            elif need <= cand1:
                st["rows_known_after_partials"] += 1
            else:
                st["rows_known_after_decision"] += 1
            if known:
                # the next decision is a known merge of the top with the element
                # below: speculate on it (its merged row P2, the row below P3)
                # instead of searching the top's row
                if L >= 3:
                    P2, P3 = self.spec_rows(t, chain[-2], chain[-3])
                else:
                    P2, P3 = (INF, -1), (INF, -1)
                st["known_spec"] += 1
                continue
            if L >= 3:
                if not pend:
                    spec = 1
                elif chain[-2] == pend[1] and t != pend[1]:
                    spec = 2
            P2y = None
            if not spec and pend and L >= 3 and self.policy == "r5c":
                spec = 4              # a merge launch whose row y is not below the top: speculate too,
                y = pend[1]           # y's own minimum kept apart (P2y) for a push of y
                m = self.active().copy()
                m[y] = False
                P2y = self.rowmin(D[y], m)
            if spec:
                P2, P3 = self.spec_rows(t, chain[-2], chain[-3])
            elif pend:
                st["m0"] += 1
                y = pend[1]
                m = self.active().copy()
                m[y] = False
                P2 = self.rowmin(D[y], m)
        return self.finish()

    def finish(self):
        n = self.n
        Z = np.array(self.Z, dtype=np.float64)
        Z = Z[np.argsort(Z[:, 2], kind="mergesort")]
        parent = np.arange(2 * n - 1)
        sz = np.ones(2 * n - 1, dtype=np.int64)

        def find(x):
            while parent[x] != x:
                parent[x] = parent[parent[x]]
                x = parent[x]
            return x
        for i in range(n - 1):
            x, y = find(int(Z[i, 0])), find(int(Z[i, 1]))
            Z[i, 0], Z[i, 1] = min(x, y), max(x, y)
            parent[x] = parent[y] = n + i
            sz[n + i] = sz[x] + sz[y]
            Z[i, 3] = sz[n + i]
        return Z


def dense_from_counts(common, n, s=1000):
    sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
    from drep_amd.d_cluster import linkage_tables
    lut, _ = linkage_tables(np.array([s]), s)
    D = np.zeros((n, n))
    iu = np.triu_indices(n, 1)
    D[iu] = lut[common]
    D.T[iu] = lut[common]
    return D, lut[common]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("counts")
    ap.add_argument("--policy", default="r4")
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--scipy", action="store_true")
    a = ap.parse_args()
    c = np.load(a.counts)
    n = int(round((1 + (1 + 8 * len(c)) ** 0.5) / 2))
    if a.n:
        # leading n x n block of the condensed triangle
        idx = np.concatenate([np.arange(i * n - i * (i + 1) // 2, i * n - i * (i + 1) // 2 + a.n - i - 1)
                              for i in range(a.n - 1)])
        n0 = n
        idx = np.concatenate([np.arange(i * n0 - i * (i + 1) // 2, i * n0 - i * (i + 1) // 2 + (a.n - i - 1))
                              for i in range(a.n - 1)])
        c = c[idx]
        n = a.n
    D, y = dense_from_counts(c, n)
    t0 = time.time()
    sim = Sim(D, a.policy)
    Z = sim.run()
    out = dict(n=n, policy=a.policy, sim_s=round(time.time() - t0, 1), **sim.stats)
    out["launches_per_merge"] = sim.stats["launches"] / (n - 1)
    if a.scipy:
        import scipy.cluster.hierarchy as sch
        Zs = sch.linkage(y, method="average")
        out["Z_identical_to_scipy"] = bool(np.array_equal(Z, Zs))
    print(out)


if __name__ == "__main__":
    main()
