from .dist import DistContext, init_distributed, init_single_rank_collective

__all__ = ["DistContext", "init_distributed", "init_single_rank_collective"]
