"""Loader for the native scheduler extension (``_sched*.so``, built in-tree by
``python -m dstack_amd.serving.build`` / ``__graft_entry__.build()``).  No Python fallback: the
engine fails loudly when the extension is missing."""

try:
    from dstack_amd.serving._sched import Scheduler  # noqa: F401
except ImportError as e:  # pragma: no cover - depends on the build
    raise ImportError("dstack_amd.serving._sched is not built: run `python -m dstack_amd.serving.build`") from e
