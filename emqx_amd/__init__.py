"""emqx_amd — MI355X-native batch topic matching for EMQX's publish routing hot path.

The compute path is libemqx_gpu_match.so (hand-written gfx950 HIP kernels behind
a C ABI, include/emqx_gpu_match.h).  This package is the host-side mirror of the
reference interfaces (emqx_topic, emqx_trie, emqx_router, emqx_broker dispatch).
"""

from ._lib import GpuMatchError, LIB_PATH  # noqa: F401
from .engine import Context, DeviceCsr, Index, gen_filter_codes, pack, render_codes  # noqa: F401
from .routing import Broker, Router, SessionRouter, Trie, default_context  # noqa: F401
from .rules import TopicRuleIndex  # noqa: F401
from . import topic  # noqa: F401

__all__ = ["Context", "Index", "DeviceCsr", "Trie", "Router", "SessionRouter", "Broker", "TopicRuleIndex", "topic",
           "GpuMatchError",
           "pack", "gen_filter_codes", "render_codes", "default_context"]
