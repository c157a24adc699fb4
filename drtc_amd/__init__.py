"""Import alias for the framework package.

The framework's source tree lives in the directory
``distributed-real-time-chat-and-collaboration-tool_amd/`` (a name that is not a
valid Python identifier).  This shim makes it importable as ``drtc_amd`` by
pointing this package's ``__path__`` at that directory and executing its
``__init__``; every submodule (``drtc_amd.ops``, ``drtc_amd.models`` ...) is
then resolved from the real tree.
"""
import os as _os

_REAL = _os.path.join(
    _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
    "distributed-real-time-chat-and-collaboration-tool_amd",
)
__path__ = [_REAL]  # noqa: F811  (submodules resolve from the real tree)
__file__ = _os.path.join(_REAL, "__init__.py")
with open(__file__, "r", encoding="utf-8") as _f:
    exec(compile(_f.read(), __file__, "exec"))
