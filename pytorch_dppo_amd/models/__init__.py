from .actor_critic import ActorCritic, LayerSpec, PackedLayout, pad32

__all__ = ["ActorCritic", "LayerSpec", "PackedLayout", "pad32"]
