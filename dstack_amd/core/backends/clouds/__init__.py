"""Cloud backends (REST, no vendor SDKs).  ``compute_class(backend_type)`` maps a backend type to
its ``Compute`` implementation."""

from __future__ import annotations

from typing import Optional, Type

from dstack_amd.core.models.backends import BackendType


def compute_class(backend_type: BackendType) -> Optional[Type]:
    from dstack_amd.core.backends.clouds import aws, containers, hyperscalers, rest_vm

    return {
        BackendType.AWS: aws.AWSCompute,
        BackendType.AZURE: hyperscalers.AzureCompute,
        BackendType.GCP: hyperscalers.GCPCompute,
        BackendType.OCI: hyperscalers.OCICompute,
        BackendType.LAMBDA: rest_vm.LambdaCompute,
        BackendType.VULTR: rest_vm.VultrCompute,
        BackendType.TENSORDOCK: rest_vm.TensorDockCompute,
        BackendType.CUDO: rest_vm.CudoCompute,
        BackendType.DATACRUNCH: rest_vm.DataCrunchCompute,
        BackendType.NEBIUS: rest_vm.NebiusCompute,
        BackendType.RUNPOD: containers.RunpodCompute,
        BackendType.VASTAI: containers.VastAICompute,
        BackendType.KUBERNETES: containers.KubernetesCompute,
    }.get(backend_type)
