"""sidekick_amd — MI355X-native quACK power-sum engine (gfx950 HIP kernels
behind the C ABI in include/quack_hip.h).  See DESIGN.md."""
from .quack import (  # noqa: F401
    CoefficientVector, Context, FlowQuacks, ModularInteger, PowerSumQuackU32, PowerSumQuackU64,
    arithmetic, device_count, get_context, roots,
)
from ._lib import P32, P64, QuackError, UndecodableError  # noqa: F401

__version__ = "0.1.0"
