"""OracleCtx -- a CPU test double of ``_lib.Context`` for the multi-rank orchestration
tests (TEST INFRASTRUCTURE: it computes every stage with the oracle, never with the
product).  It implements exactly the methods ``sharded.run_sharded`` calls, with the
device's data contract (squared distances as float32, global trainIdx, partial
histograms over owned votes, first-touch ordinals q*16+slot)."""
import numpy as np

from oracle import oracle as orc


class OracleCtx:
    def __init__(self, db, lo, hi, qdes, qkp, bins=None):
        self.db, self.lo, self.hi = db, lo, hi
        self.qdes = np.asarray(qdes)
        self.qkp = qkp
        self.nq = len(self.qdes)

    # ---- match ----
    def match(self):
        q = self.qdes.astype(np.int64)
        d = self.db.des[self.lo:self.hi].astype(np.int64)
        sq = ((q[:, None, :] - d[None, :, :]) ** 2).sum(-1).astype(np.float32)
        best = np.argmin(sq, axis=1)
        r = np.arange(self.nq)
        self.cd1 = sq[r, best].copy()
        self.cidx = (best + self.lo).astype(np.int32)
        sq[r, best] = np.inf
        self.cd2 = sq.min(axis=1) if sq.shape[1] > 1 else np.full(self.nq, np.inf, np.float32)

    def candidates(self):
        return self.cd1.copy(), self.cidx.copy(), self.cd2.copy()

    def merge_candidates(self, g1, gi, g2):
        P = len(g1) // self.nq
        g1, gi, g2 = (a.reshape(P, self.nq) for a in (g1, gi, g2))
        v1, i1, v2 = g1[0].copy(), gi[0].copy(), g2[0].copy()
        for p in range(1, P):
            better = (g1[p] < v1) | ((g1[p] == v1) & (gi[p] < i1))
            nv2 = np.where(better, np.minimum(v1, g2[p]), np.minimum(v2, g1[p]))
            v1 = np.where(better, g1[p], v1)
            i1 = np.where(better, gi[p], i1)
            v2 = nv2
        self.cd1, self.cidx, self.cd2 = v1, i1, v2

    def ratio(self, ratio=0.75):
        self.d1 = np.sqrt(self.cd1, dtype=np.float32)
        self.d2 = np.sqrt(self.cd2, dtype=np.float32)
        self.idx1 = self.cidx
        self.good = orc.ratio_test(self.d1, self.d2, ratio)

    def match_result(self):
        return self.idx1, self.d1, self.d2, self.good

    # ---- hough ----
    def hough(self, shape, bins, own):
        self.shape = shape
        self.bins = orc._bins4(bins)
        bx, by, bt, bs = self.bins
        dbkp = {"x": self.db.kp.x, "y": self.db.kp.y, "angle": self.db.kp.angle,
                "octave": self.db.kp.octave, "img": self.db.img}
        qkp = {"x": self.qkp.x, "y": self.qkp.y, "angle": self.qkp.angle,
               "octave": self.qkp.octave}
        self._dbkp, self._qkp = dbkp, qkp
        nb = bx * by * bt * bs
        self.counts = np.zeros(nb, np.uint32)
        self.first = np.full(nb, 0xFFFFFFFF, np.uint32)
        self.votes = {}     # q -> list of (slot, lin)
        for q in np.nonzero(self.good)[0]:
            m = int(self.idx1[q])
            pose = orc.match_poses([(int(q), m)], qkp, dbkp,
                                   {"centroid": self.db.centroid, "size": self.db.size})[0]
            ix, iy, it, isg = orc.calculate_bin_index(pose, self.bins, shape)
            vl = []
            for slot in range(16):
                w, x, y, z = (slot >> 3) & 1, (slot >> 2) & 1, (slot >> 1) & 1, slot & 1
                k = (ix + w, iy + x, it + y, isg + z)
                if k[0] < bx and k[1] < by and k[2] < bt and k[3] < bs:
                    lin = ((k[0] * by + k[1]) * bt + k[2]) * bs + k[3]
                    vl.append((slot, lin))
                    if own[0] <= m < own[1]:
                        self.counts[lin] += 1
                        self.first[lin] = min(self.first[lin], q * 16 + slot)
            self.votes[int(q)] = vl

    def hough_partial(self):
        return self.counts.copy(), self.first.copy()

    def set_hough_partial(self, counts, first):
        self.counts, self.first = counts.astype(np.uint32), first.astype(np.uint32)

    def select(self, thr):
        valid = [lin for lin in range(len(self.counts))
                 if self.counts[lin] >= max(thr, 1)]
        valid.sort(key=lambda lin: self.first[lin])
        bx, by, bt, bs = self.bins
        keys, members, off = [], [], [0]
        for lin in valid:
            keys.append((lin // (bs * bt * by), (lin // (bs * bt)) % by, (lin // bs) % bt, lin % bs))
            mem = [q for q in sorted(self.votes) if any(l == lin for _, l in self.votes[q])]
            members.extend(mem)
            off.append(len(members))
        self.valid = {"keys": np.array(keys, np.int32).reshape(-1, 4),
                      "votes": np.diff(off).astype(np.int32),
                      "offsets": np.array(off, np.int64),
                      "members": np.array(members, np.int32)}

    def valid_result(self):
        return self.valid

    def affine(self, size, xf, yf, thr):
        res = []
        v = self.valid
        for i in range(len(v["keys"])):
            b = orc.OBin(tuple(int(k) for k in v["keys"][i]), (0, 0), None, (0, 0, 0, 0))
            b.members = [(int(q), int(self.idx1[q])) for q in
                         v["members"][v["offsets"][i]:v["offsets"][i + 1]]]
            b.votes = len(b.members)
            res.append(b)
        self.aff = orc.affine_verify(res, self._qkp, self._dbkp, size, thr)

    def affine_result(self):
        return self.aff
