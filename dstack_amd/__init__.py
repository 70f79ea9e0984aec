"""dstack_amd — an MI355X-native AI-workload orchestrator with dstack's capabilities.

Layers (see SURVEY.md §1 for the reference layer map this mirrors):

* ``dstack_amd.core``      — pydantic domain models (YAML configs, runs, fleets, ...), SSH, backends.
* ``dstack_amd.server``    — control-plane server (FastAPI + SQLite), event-driven reconcilers.
* ``dstack_amd.proxy``     — gateway app, service/model (OpenAI) proxy.
* ``dstack_amd.cli`` / ``dstack_amd.api`` — the ``dstack`` CLI and Python API.
* ``native/``              — C++ ``dstack-runner`` / ``dstack-shim`` agents and HIP probes.
* ``dstack_amd.models`` / ``ops`` / ``parallel`` — the MI355X training workload the orchestrator
  runs and benchmarks (Llama-3 on hand-written HIP/CDNA4 kernels, ZeRO-1 DP over RCCL).
"""

__version__ = "0.1.0"
