"""MI355X-native flip-walk engine for connected graph partitions.

A from-scratch HIP/gfx950 implementation of the hot path of
LorenzoNajt/FlipComplexityEmpirical (``grid_chain_sec11.py`` / ``Frankenstein_chain.py``):
the k=2 single-node-flip Markov chain driven through gerrychain's ``MarkovChain`` with
``slow_reversible_propose_bi``, ``single_flip_contiguous`` + population bound and the
``cut_accept`` Metropolis rule, plus the driver's per-step diagnostics.

Layers:
  graphs       host-side lattice / plan builders (networkx -> CSR + positions)
  engine       FlipGraph / FlipRun over the C-ABI of libflipchain.so
  chain        gerrychain-shaped drop-in API (Partition, MarkovChain, Validator, ...)
  distributed  chain sharding over GPUs + RCCL reduction of statistics
"""
from .graphs import GraphSpec  # noqa: F401

__all__ = ["GraphSpec"]
