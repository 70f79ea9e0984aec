"""Error hierarchy shared by the server, CLI and API (reference: ``C/errors.py:5-134``)."""

from __future__ import annotations

from typing import List, Optional


class DstackError(Exception):
    pass


class ConfigurationError(DstackError):
    pass


class CLIError(DstackError):
    pass


class ServerError(DstackError):
    pass


class ServerClientErrorCode:
    UNSPECIFIED_ERROR = "error"
    RESOURCE_EXISTS = "resource_exists"
    RESOURCE_NOT_EXISTS = "resource_not_exists"
    FORBIDDEN = "forbidden"
    UNAUTHORIZED = "unauthorized"
    INVALID_REQUEST = "invalid_request"
    BACKEND_NOT_AVAILABLE = "backend_not_available"
    RESOURCE_BUSY = "resource_busy"
    INVALID_CREDENTIALS = "invalid_credentials"


class ServerClientError(ServerError):
    """An error the server reports to the client with HTTP 400."""

    code: str = ServerClientErrorCode.UNSPECIFIED_ERROR
    msg: str = ""

    def __init__(self, msg: Optional[str] = None, fields: Optional[List[List[str]]] = None):
        self.msg = msg if msg is not None else self.msg
        self.fields = fields or []
        super().__init__(self.msg)


class ResourceExistsError(ServerClientError):
    code = ServerClientErrorCode.RESOURCE_EXISTS
    msg = "Resource exists"


class ResourceNotExistsError(ServerClientError):
    code = ServerClientErrorCode.RESOURCE_NOT_EXISTS
    msg = "Resource not found"


class ForbiddenError(ServerClientError):
    code = ServerClientErrorCode.FORBIDDEN
    msg = "Access denied"


class UnauthorizedError(ServerClientError):
    code = ServerClientErrorCode.UNAUTHORIZED
    msg = "Unauthorized"


class InvalidRequestError(ServerClientError):
    code = ServerClientErrorCode.INVALID_REQUEST


class BackendNotAvailable(ServerClientError):
    code = ServerClientErrorCode.BACKEND_NOT_AVAILABLE
    msg = "Backend not available"


class RepoDoesNotExistError(ServerClientError):
    code = ServerClientErrorCode.RESOURCE_NOT_EXISTS
    msg = "Repo does not exist"


class ResourceBusyError(ServerClientError):
    """A resource is locked by another operation (a reconciler pass, a concurrent request) for
    longer than the caller waits: transient, retry (HTTP 409 on the API; background callers retry
    on their next pass instead of failing the job)."""

    code = ServerClientErrorCode.RESOURCE_BUSY
    msg = "Resource is being processed, retry"


class InvalidCredentialsError(ServerClientError):
    """Backend credentials the cloud rejected (reference ``BackendInvalidCredentialsError``,
    ``S/services/backends/configurators/*``)."""

    code = ServerClientErrorCode.INVALID_CREDENTIALS
    msg = "Invalid credentials"


class GatewayError(ServerClientError):
    msg = "Gateway error"


class BackendError(DstackError):
    pass


class BackendInvalidCredentialsError(BackendError):
    pass


class BackendAuthError(BackendError):
    pass


class ComputeError(BackendError):
    pass


class NoCapacityError(ComputeError):
    pass


class ProvisioningError(ComputeError):
    pass


class ComputeResourceNotFoundError(ComputeError):
    pass


class PlacementGroupInUseError(ComputeError):
    pass


class NotYetTerminated(ComputeError):
    """The resource termination is in progress; retry later."""


class SSHError(DstackError):
    pass


class SSHTimeoutError(SSHError):
    pass


class SSHConnectionRefusedError(SSHError):
    pass


class SSHKeyError(SSHError):
    pass


class SSHPortInUseError(SSHError):
    pass


class RunnerError(DstackError):
    """The in-container agent (dstack-runner) or host agent (dstack-shim) failed a request."""


class ClientError(DstackError):
    """Client-side failure talking to the server (reference: ``core/errors.py`` ``ClientError``)."""


class URLNotFoundError(ClientError):
    pass


class MethodNotAllowedError(ClientError):
    pass


class DockerRegistryError(DstackError):
    """The registry answered, and not with the image's config (unknown image or tag, no access,
    malformed or oversized config); ``status`` is the HTTP status when there was one."""

    def __init__(self, msg: str = "", status: int = 0):
        super().__init__(msg)
        self.status = status
