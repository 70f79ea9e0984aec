"""Profile parameters shared by run/fleet configurations and ``profiles.yml`` (reference:
``C/models/profiles.py:115-257``)."""

from __future__ import annotations

from enum import Enum
from typing import List, Literal, Optional, Union

from pydantic import Field, field_validator, model_validator

from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.common import CoreModel, Duration

DEFAULT_RETRY_DURATION = 3600
DEFAULT_POOL_NAME = "default-pool"
DEFAULT_RUN_TERMINATION_IDLE_TIME = 5 * 60
DEFAULT_FLEET_TERMINATION_IDLE_TIME = 72 * 60 * 60
DEFAULT_INSTANCE_RETRY_DURATION = 60 * 60 * 24
DEFAULT_STOP_DURATION = 300


class SpotPolicy(str, Enum):
    SPOT = "spot"
    ONDEMAND = "on-demand"
    AUTO = "auto"


class CreationPolicy(str, Enum):
    REUSE = "reuse"
    REUSE_OR_CREATE = "reuse-or-create"


class TerminationPolicy(str, Enum):
    DONT_DESTROY = "dont-destroy"
    DESTROY_AFTER_IDLE = "destroy-after-idle"


class RetryEvent(str, Enum):
    NO_CAPACITY = "no-capacity"
    INTERRUPTION = "interruption"
    ERROR = "error"


def parse_duration(v):
    if v is None:
        return None
    return Duration.parse(v)


def parse_off_duration(v):
    """``off``/``false`` → "off"; ``true`` → None (default); else seconds."""
    if v == "off" or v is False:
        return "off"
    if v is True:
        return None
    return parse_duration(v)


def parse_idle_duration(v):
    if v == "off" or v is False:
        return -1
    if v is True:
        return None
    return parse_duration(v)


class ProfileRetryPolicy(CoreModel):
    """Deprecated form of ``retry``."""

    retry: bool = False
    duration: Optional[Union[int, str]] = None

    @field_validator("duration", mode="before")
    @classmethod
    def _d(cls, v):
        return parse_duration(v)

    @model_validator(mode="after")
    def _fill(self):
        if self.retry and self.duration is None:
            self.duration = DEFAULT_RETRY_DURATION
        if self.duration is not None:
            self.retry = True
        return self


class ProfileRetry(CoreModel):
    on_events: List[RetryEvent]
    duration: Optional[Union[int, str]] = None

    @field_validator("duration", mode="before")
    @classmethod
    def _d(cls, v):
        return parse_duration(v)

    @model_validator(mode="after")
    def _check(self):
        if len(self.on_events) == 0:
            raise ValueError("`on_events` cannot be empty")
        return self


class ProfileParams(CoreModel):
    backends: Optional[List[BackendType]] = Field(None, description="Backends to consider, e.g. [remote, aws]")
    regions: Optional[List[str]] = None
    instance_types: Optional[List[str]] = None
    reservation: Optional[str] = None
    spot_policy: Optional[SpotPolicy] = None
    retry: Optional[Union[ProfileRetry, bool]] = None
    max_duration: Optional[Union[Literal["off"], str, int, bool]] = None
    stop_duration: Optional[Union[Literal["off"], str, int, bool]] = None
    max_price: Optional[float] = Field(None, gt=0.0)
    creation_policy: Optional[CreationPolicy] = None
    idle_duration: Optional[Union[Literal["off"], str, int, bool]] = None
    # deprecated
    termination_policy: Optional[TerminationPolicy] = None
    termination_idle_time: Optional[Union[str, int]] = None
    pool_name: Optional[str] = None
    instance_name: Optional[str] = None
    retry_policy: Optional[ProfileRetryPolicy] = None

    @field_validator("max_duration", "stop_duration", mode="before")
    @classmethod
    def _off(cls, v):
        return parse_off_duration(v)

    @field_validator("idle_duration", mode="before")
    @classmethod
    def _idle(cls, v):
        return parse_idle_duration(v)

    @field_validator("termination_idle_time", mode="before")
    @classmethod
    def _tit(cls, v):
        return parse_duration(v)


PROFILE_PARAM_NAMES = list(ProfileParams.model_fields)


class Profile(ProfileParams):
    name: str = Field(..., description="Profile name, usable as --profile")
    default: bool = False


class ProfilesConfig(CoreModel):
    profiles: List[Profile]

    def default(self) -> Optional[Profile]:
        for p in self.profiles:
            if p.default:
                return p
        return None

    def get(self, name: str) -> Profile:
        for p in self.profiles:
            if p.name == name:
                return p
        raise KeyError(name)
