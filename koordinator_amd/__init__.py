"""koordinator_amd — MI355X batch Filter/Score engine for koord-scheduler (NodeResourcesFit + LoadAwareScheduling).

The compute path is libkoordgpu.so (HIP/gfx950 kernels + C++ host runtime, C ABI in include/koordgpu.h);
this package is the Python host layer over that ABI.  There is no CPU fallback: if the library is missing
every entry point raises.
"""
from . import abi  # noqa: F401
from .engine import Engine, default_config  # noqa: F401
from .framework import (LoadAwareSchedulingArgs, NodeResourcesFitArgs, Profile, Scheduler,  # noqa: F401
                        build_config, make_node, make_node_metric, make_pod)
