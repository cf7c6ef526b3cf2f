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

    def __init__(self, k, n_kmers=1 << 10, max_kmers=1 << 24):
        self.k = k
        self.n_kmers = n_kmers
        self.max_kmers = max_kmers
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

    def route_win(self, recs, nranks, words, win):
        """The one-pass route's layout (kh_route_starts_win_dev): owner q's words in the window at
        words[q * win * W ...]; enabled per instance with route_windows = True."""
        enc, counts = self.route(recs, nranks, starts=True)
        pos = 0
        for q in range(nranks):
            c = int(counts[q])
            words[q * win * self.W:(q * win + c) * self.W].copy_(enc[pos * self.W:(pos + c) * self.W])
            pos += c
        return counts

    def reserve(self, m):
        """kh_reserve: the shard grows to what it receives (fails like the GPU on NOMEM)."""
        if m > self.max_kmers:
            raise RuntimeError(f"shard cannot hold {m} k-mers")
        self.n_kmers = max(self.n_kmers, m)

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

    # -- migrating walkers (same contract as kh_mwalk_*; messages and records are opaque words) --
    MSG_WORDS = 5
    TEXT_REC_WORDS = 2

    def zeros(self, n, dtype):
        return torch.zeros(max(int(n), 1), dtype=dtype)

    def counters(self):
        return torch.tensor([len(self.starts), 0], dtype=torch.int64)

    def route_splitters(self, nranks):
        return torch.zeros(nranks, dtype=torch.int64)   # no splitter segments in the double

    def mw_begin(self, nranks, rank, total_kmers, n_starts, n_splitters, total_walkers):
        assert n_starts == len(self.starts)
        self.nranks, self.rank = nranks, rank
        self.store = []                                    # (origin, fin, pos, idx, value)
        self.first = True
        self.carry = []                                    # (owner, message) held back
        return len(self.starts)

    def _msg(self, key, fwd, steps, idx, origin):
        kw = self._enc([key]).numpy()[:2]
        return [int(kw[0]), int(kw[1]), steps, idx, origin | (fwd << 8)]

    def mw_round(self, inp, cap_in, out, cap_out, live):
        """kh_mwalk_round_dev: P slots in (None: this rank's starts), P slots of cap_out out,
        messages past a slot's capacity held back for the next round; live = [in flight, largest
        per-destination count]."""
        P = self.nranks
        if self.first:
            msgs = [self._msg(s[:self.P], s[self.P + 1], 0, i, self.rank) for i, s in enumerate(self.starts)]
            self.first = False
        else:
            a = inp.numpy()
            sw = 2 + cap_in * 5
            msgs = []
            for q in range(P):
                c = int(a[q * sw])
                for i in range(c):
                    msgs.append(list(map(int, a[q * sw + 2 + 5 * i:q * sw + 7 + 5 * i])))
        outs = list(self.carry)
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
        o = out.numpy()
        sw = 2 + cap_out * 5
        counts = [0] * P
        self.carry = []
        for q, m in outs:
            if counts[q] < cap_out:
                o[q * sw + 2 + 5 * counts[q]:q * sw + 7 + 5 * counts[q]] = m
                counts[q] += 1
            else:
                self.carry.append((q, m))
        per = [0] * P
        for q, _ in outs:
            per[q] += 1
        for q in range(P):
            o[q * sw] = counts[q]
            o[q * sw + 1] = 0
        live[0] = len(outs)
        live[1] = max(per) if per else 0

    def mw_text_bound(self):
        return len(self.store)

    def _rec_words(self, r):
        origin, fin, pos, idx, val = r
        return [(origin << 56) | (fin << 55) | (pos << 31) | idx, val]

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

    def sync(self):
        pass

    def contigs_text(self):
        return self.text
