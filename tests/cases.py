"""Shared generators of edge-case inputs (test infrastructure; no GPU, no product imports)."""
import numpy as np


def merging_walks_text(k, L, seed, every=1):
    """Malformed input whose start walks overlap: one chain C_0..C_{L-1} plus, at every `every`-th
    position j, three extra start k-mers x + C_{j-1}[1:] (bwd 'F') whose next_kmer is C_j. Every
    start walks the shared tail again (kmer_hash.cpp:41-53 does not care), so the text is ~3L^2/2
    bases, far past the table-start bound n + (K+1)·starts that kh_assemble_dev sizes first.
    Returns the fixed-width text (read_kmers.hpp:54-79 lines)."""
    rng = np.random.default_rng(seed)
    B = "ACGT"
    seq = "".join(B[x] for x in rng.integers(0, 4, L + k - 1))
    lines = []
    for i in range(L):
        lines.append((seq[i:i + k], "F" if i == 0 else seq[i - 1], "F" if i == L - 1 else seq[i + k]))
    seen = {x[0] for x in lines}
    for j in range(1, L, every):
        for x in B:
            z = x + seq[j:j + k - 1]
            if x == seq[j - 1] or z in seen:
                continue
            seen.add(z)
            lines.append((z, "F", seq[j + k - 1]))
    order = rng.permutation(len(lines))
    return "".join(f"{lines[i][0]} {lines[i][1]}{lines[i][2]}\n" for i in order).encode()
