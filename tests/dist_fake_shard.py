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

    def __init__(self, k, n_kmers=1 << 24):
        self.k = k
        self.n_kmers = n_kmers
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

    def route(self, recs, nranks, words=None, starts=False):
        if starts:
            self.collect_starts(recs)
        rows = [bytes(r) for r in recs.numpy()]
        payloads, _, counts = self._group([(self._owner(r[:self.P], nranks), r) for r in rows], nranks)
        enc = self._enc(payloads)
        if words is not None:  # caller's buffer (the pipelined insert routes into slices of one)
            words[:min(words.numel(), enc.numel())].copy_(enc[:words.numel()])
            return words, counts
        return enc, counts

    def insert_words(self, words, m):
        for rec in self._dec(words, m, self.R):
            assert rec[:self.P] not in self.table, "duplicate k-mer"
            self.table[rec[:self.P]] = rec

    # staged insert (kh_insert_words_stage_dev / _finish): chunks are kept until finish
    def stage_words(self, words, m, total):
        self.staged = getattr(self, "staged", [])
        self.staged.append(words[:m * 2].clone())
        assert sum(t.numel() // 2 for t in self.staged) <= total

    def finish_words(self):
        for t in getattr(self, "staged", []):
            self.insert_words(t, t.numel() // 2)
        self.staged = []

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

    # -- migrating walkers (same contract as kh_mwalk_*; messages and records are opaque words) --
    MSG_WORDS = 5
    TEXT_REC_WORDS = 2

    def zeros(self, n, dtype):
        return torch.zeros(max(int(n), 1), dtype=dtype)

    def mw_begin(self, nranks, rank, total_kmers):
        self.nranks, self.rank = nranks, rank
        self.store = []                                    # (origin, fin, pos, idx, value)
        self.first = True
        return len(self.starts)

    def _msg(self, key, fwd, steps, idx, origin):
        kw = self._enc([key]).numpy()[:2]
        return [int(kw[0]), int(kw[1]), steps, idx, origin | (fwd << 8)]

    def mw_round(self, inp, n_in, out):
        if self.first:
            msgs = [self._msg(s[:self.P], s[self.P + 1], 0, i, self.rank) for i, s in enumerate(self.starts)]
            self.first = False
        else:
            a = inp[:n_in * 5].numpy().reshape(n_in, 5)
            msgs = [list(map(int, r)) for r in a]
        outs = []
        for m in msgs:
            key = bytes(np.array(m[:2], np.int64).view(np.uint8)[:self.P])
            steps, idx, origin, fwd = m[2], m[3], m[4] & 0xFF, (m[4] >> 8) & 0xFF
            if fwd == 0xFF:                                # look the key up here (its owner)
                rec = self.table.get(key)
                if rec is None:
                    raise RuntimeError("Error: k-mer not found in Distributed HashMap.")
                fwd = rec[self.P + 1]
            while True:
                if fwd == ord("F"):
                    self.store.append((origin, 1, 0, idx, steps))
                    break
                self.store.append((origin, 0, steps, idx, fwd))   # base `steps` of the contig
                steps += 1
                rec = np.frombuffer(key + b"X" + bytes([fwd]), np.uint8)
                key = bytes(ob.next_kmer(self.k, rec))     # kmer_t.hpp:51-53
                q = self._owner(key, self.nranks)
                if q != self.rank:
                    outs.append((q, self._msg(key, 0xFF, steps, idx, origin)))
                    break
                rec = self.table.get(key)
                if rec is None:
                    raise RuntimeError("Error: k-mer not found in Distributed HashMap.")
                fwd = rec[self.P + 1]
        outs.sort(key=lambda x: x[0])
        o = out.numpy()
        for j, (_, m) in enumerate(outs):
            o[j * 5:(j + 1) * 5] = m
        counts = np.zeros(self.nranks + 1, np.int64)
        for q, _ in outs:
            counts[q] += 1
        counts[self.nranks] = len(outs)
        return torch.from_numpy(counts)

    def _rec_words(self, r):
        origin, fin, pos, idx, val = r
        return [(origin << 56) | (fin << 55) | (pos << 31) | idx, val]

    def mw_text_count(self):
        return len(self.store)

    def mw_text(self, out):
        recs = sorted(self.store, key=lambda r: r[0])
        o = out.numpy()
        for j, r in enumerate(recs):
            w = self._rec_words(r)
            o[2 * j], o[2 * j + 1] = w                     # origin < 64: tag < 2^62
        counts = np.zeros(self.nranks + 1, np.int64)
        for r in recs:
            counts[r[0]] += 1
        counts[self.nranks] = len(recs)
        return torch.from_numpy(counts)

    def mw_end(self, recs, n):
        a = recs[:2 * n].numpy().view(np.uint64).reshape(n, 2) if n else np.zeros((0, 2), np.uint64)
        lens, bases = {}, {}
        for t, v in a:
            t, v = int(t), int(v)
            idx, pos, fin = t & 0x7FFFFFFF, (t >> 31) & 0xFFFFFF, (t >> 55) & 1
            if fin:
                lens[idx] = v
            else:
                bases[(idx, pos)] = chr(v)
        out = []
        for i, s in enumerate(self.starts):
            assert i in lens, "walker did not come home"
            head = ob.unpack(self.k, np.frombuffer(s[:self.P], np.uint8))
            out.append(head + "".join(bases[(i, j)] for j in range(lens[i])) + "\n")
        self.text = "".join(out).encode()

    def walk_end(self):
        self.text = "".join(w[2] + "\n" for w in self.walkers).encode()

    def sync(self):
        pass

    def contigs_text(self):
        return self.text
