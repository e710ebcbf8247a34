"""SNP-block sharding of the GRM across ranks.

K = sum_b Z_b Z_b^T over SNP blocks b (snpreader.py:651-655), so blocks can be summed in
any grouping: rank r takes blocks r, r+p, r+2p, ... (round-robin keeps the ranks within
one block of each other), accumulates a partial K in HBM, and one all-reduce(sum) of the
upper-triangle K tiles over xGMI (RCCL) yields K on every rank.  Stats per block are local
and are gathered in block order (Unit._merge_trained, unit.py:53-56).
"""


def snp_blocks(n_sid, block_size):
    """[(start, count)] covering range(n_sid) in blocks of ``block_size``."""
    block_size = max(1, int(block_size))
    return [(s0, min(block_size, n_sid - s0)) for s0 in range(0, n_sid, block_size)]


def rank_blocks(n_sid, block_size, rank, world):
    """The blocks rank ``rank`` of ``world`` owns (round-robin)."""
    assert 0 <= rank < world
    return snp_blocks(n_sid, block_size)[rank::world]


def merge_order(n_sid, block_size, world):
    """For each global block (in SNP order): (owner rank, index within that rank's list)."""
    out = []
    for b, _ in enumerate(snp_blocks(n_sid, block_size)):
        out.append((b % world, b // world))
    return out
