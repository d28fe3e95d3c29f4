"""mazero_amd — MI355X-native batched sampled-MCTS planning loop for MAZero (RDG0818/MAZero).

The hot path -- per-simulation select / expand / back-propagate over many independent roots --
runs in hand-written HIP kernels for gfx950 (mazero_amd/csrc/mzmcts.hip) behind the C-ABI of
include/mzmcts.h.  Python surfaces:

  mazero_amd.cytree.Tree_batch        drop-in for core.mcts.ctree.ctree_sampled.cytree.Tree_batch
  mazero_amd.mcts_sampled.SampledMCTS drop-in for core.mcts.tree_search.SampledMCTS (device loop)
"""
__all__ = ["cytree"]
