"""CPU test double of cs267_hw3_amd.dist.GpuShard — TEST INFRASTRUCTURE ONLY.

Implements the per-rank local operations with Python dicts and the oracle's codec (string-round-trip
next_kmer, djb2 owner), so the SPMD driver's routing, count exchange, round structure and
termination are exercised over a real torch.distributed gloo group with no GPU.
"""
import numpy as np
import torch

import oracle_bind as ob


class FakeShard:
    W = 2  # 16 bytes per routed record / query key

    def __init__(self, k):
        self.k = k
        self.P = (k + 3) // 4
        self.R = self.P + 2
        assert self.R <= 16
        self.clear()

    # -- helpers ------------------------------------------------------------------------------
    def _enc(self, rows):
        """list of <=16-byte strings -> int64 tensor [len * 2]."""
        buf = np.zeros((max(len(rows), 1), 16), np.uint8)
        for i, r in enumerate(rows):
            buf[i, :len(r)] = np.frombuffer(r, np.uint8)
        return torch.from_numpy(buf.view(np.int64).reshape(-1).copy())

    def _dec(self, t, m, width):
        a = t[:m * 2].numpy().view(np.uint8).reshape(m, 16)
        return [bytes(a[i, :width]) for i in range(m)]

    def _owner(self, key, nranks):
        return ob.djb2(self.k, np.frombuffer(key, np.uint8)) % nranks

    def _group(self, items, nranks):
        """items: list of (owner, payload) -> (payloads in owner order, counts tensor [P+1])."""
        order = sorted(range(len(items)), key=lambda i: items[i][0])
        counts = np.zeros(nranks + 1, np.int64)
        for q, _ in items:
            counts[q] += 1
        counts[nranks] = len(items)
        return [items[i][1] for i in order], order, torch.from_numpy(counts)

    # -- shard interface --------------------------------------------------------------------------
    def clear(self):
        self.table = {}
        self.starts = []

    def collect_starts(self, recs):
        for r in recs.numpy():
            if r[self.P] == ord("F"):
                self.starts.append(bytes(r))

    def route(self, recs, nranks):
        rows = [bytes(r) for r in recs.numpy()]
        payloads, _, counts = self._group([(self._owner(r[:self.P], nranks), r) for r in rows], nranks)
        return self._enc(payloads), counts

    def insert_words(self, words, m):
        for rec in self._dec(words, m, self.R):
            assert rec[:self.P] not in self.table, "duplicate k-mer"
            self.table[rec[:self.P]] = rec

    def walk_begin(self, total_kmers):
        # walker = [key bytes, fwd char (None = query in flight), contig string, done, reply pos]
        self.walkers = []
        for s in self.starts:
            self.walkers.append([s[:self.P], chr(s[self.P + 1]),
                                 ob.unpack(self.k, np.frombuffer(s[:self.P], np.uint8)), False, -1])
        self.nw = len(self.walkers)
        return self.nw

    def walk_emit(self, nranks):
        items = []
        for i, w in enumerate(self.walkers):
            if w[3]:
                continue
            if w[1] == "F":
                w[3] = True
                continue
            w[2] += w[1]                                   # extract_contig appends fwd ext
            rec = np.frombuffer(w[0] + b"X" + w[1].encode(), np.uint8)
            w[0] = bytes(ob.next_kmer(self.k, rec))        # kmer_t.hpp:51-53
            items.append((self._owner(w[0], nranks), (i, w[0])))
        payloads, _, counts = self._group(items, nranks)
        self.qperm = [p[0] for p in payloads]
        return self._enc([p[1] for p in payloads]), counts

    def find_ext(self, keys, m):
        out = np.full(max(m, 1), 0xFF, np.uint8)
        for j, key in enumerate(self._dec(keys, m, self.P)):
            rec = self.table.get(key)
            if rec is not None:
                out[j] = rec[self.P + 1]                   # forward extension char
        return torch.from_numpy(out)

    def walk_apply(self, ext, m):
        e = ext[:m].numpy()
        for j in range(m):
            w = self.walkers[self.qperm[j]]
            if e[j] == 0xFF:
                raise RuntimeError("Error: k-mer not found in Distributed HashMap.")
            w[1] = chr(e[j])

    # -- fixed-capacity rounds (same contract as kh_walk_emit_fixed_dev & co.) ------------------
    S = 8  # KH_SEG_SUBS

    def step_fixed(self, nranks, cap, reply_prev, send):
        """Apply the previous round's replies (walker.pos -> reply_prev index), then emit.
        Walker i fills sub-segment i % S (the GPU uses its block's index)."""
        S, C8 = self.S, cap // self.S
        L = S + cap * self.W
        cursors = [[0] * S for _ in range(nranks)]
        sv = send.numpy()
        rp = reply_prev.numpy() if reply_prev is not None else None
        for i, w in enumerate(self.walkers):
            if w[3]:
                continue
            if w[1] is None:                               # query in flight
                r = rp[w[4]]
                if r == 0xFF:
                    raise RuntimeError("Error: k-mer not found in Distributed HashMap.")
                w[1] = chr(r)
            if w[1] == "F":
                w[3] = True
                continue
            rec = np.frombuffer(w[0] + b"X" + w[1].encode(), np.uint8)
            nk = bytes(ob.next_kmer(self.k, rec))          # kmer_t.hpp:51-53
            q, x = self._owner(nk, nranks), i % S
            if cursors[q][x] >= C8:
                continue                                   # sub-segment full: retry next round
            slot = x * C8 + cursors[q][x]
            cursors[q][x] += 1
            w[2] += w[1]                                   # extract_contig appends fwd ext
            w[0] = nk
            w[1] = None
            w[4] = q * cap + slot
            sv[q * L + S + slot * 2:q * L + S + 2 + slot * 2] = self._enc([nk]).numpy()[:2]
        for q in range(nranks):
            sv[q * L:q * L + S] = cursors[q]

    def find_ext_fixed(self, nranks, cap, recv, reply):
        S, C8 = self.S, cap // self.S
        L = S + cap * self.W
        rv = recv.numpy()
        out = reply.numpy()
        for q in range(nranks):
            for x in range(S):
                m = int(rv[q * L + x])
                b = q * L + S + x * C8 * 2
                keys = self._dec(torch.from_numpy(rv[b:b + m * 2].copy()), m, self.P)
                for j, key in enumerate(keys):
                    rec = self.table.get(key)
                    out[q * cap + x * C8 + j] = rec[self.P + 1] if rec is not None else 0xFF

    def active(self):
        return torch.tensor([sum(not w[3] for w in self.walkers)], dtype=torch.int64)

    def walk_end(self):
        self.text = "".join(w[2] + "\n" for w in self.walkers).encode()

    def sync(self):
        pass

    def contigs_text(self):
        return self.text
