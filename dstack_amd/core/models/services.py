"""Service-run data structures: the OpenAI-compatible model mapping (reference:
``C/models/services.py``) and autoscaling specs."""

from __future__ import annotations

from typing import Literal, Optional, Union

from pydantic import Field
from typing_extensions import Annotated

from dstack_amd.core.models.common import CoreModel, Duration


class BaseChatModel(CoreModel):
    type: Literal["chat"] = "chat"
    name: str
    format: str


class TGIChatModel(BaseChatModel):
    format: Literal["tgi"]
    chat_template: Optional[str] = None
    eos_token: Optional[str] = None


class OpenAIChatModel(BaseChatModel):
    format: Literal["openai"]
    prefix: str = "/v1"


ChatModel = Annotated[Union[TGIChatModel, OpenAIChatModel], Field(discriminator="format")]
AnyModel = ChatModel


class ScalingSpec(CoreModel):
    """Autoscaling rule.  ``rps`` = requests/s per replica (gateway stats); ``gpu_util`` = mean
    amdsmi GPU busy % across a replica's GPUs (MI355X addition: scale LLM serving on the
    accelerator saturation rather than on request rate)."""

    metric: Literal["rps", "gpu_util"]
    target: float
    scale_up_delay: Duration = Duration.parse("5m")
    scale_down_delay: Duration = Duration.parse("10m")
