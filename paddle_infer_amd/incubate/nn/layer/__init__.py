from .fused_transformer import *  # noqa: F401,F403
