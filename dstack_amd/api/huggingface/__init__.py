"""Hugging Face task builders (reference: ``src/dstack/api/huggingface/__init__.py:6-73``).

``SFTFineTuningTask`` is a ready-made :class:`~dstack_amd.api.Task`: LoRA supervised fine-tuning of a
Hub model on a Hub dataset with transformers + peft + trl, on the default ROCm PyTorch image.  The
training script (``sft_train.py`` next to this file) travels inside the task's commands, so the task
needs no repo.  With several GPUs it runs under ``accelerate launch`` -- one process per GPU over
RCCL.  MI355X differences from the reference's defaults: bf16 compute and a bf16 base (288 GB of HBM
per GPU hold the unquantised model); ``use_4bit=True`` still works through bitsandbytes' ROCm backend.

    task = SFTFineTuningTask(model_name="meta-llama/Llama-3.1-8B", dataset_name="org/chat-sft",
                             env={"HF_TOKEN": token}, resources=Resources(gpu="MI355X:8"))
    client.runs.apply_configuration(task)
"""

from __future__ import annotations

import base64
import shlex
from pathlib import Path
from typing import Dict, Optional

from dstack_amd.core.models.configurations import TaskConfiguration

_SCRIPT = Path(__file__).with_name("sft_train.py")
_SCRIPT_PATH = "/tmp/dstack_sft_train.py"
_PIP = "pip install --no-cache-dir --quiet 'transformers>=4.44' 'peft>=0.12' 'trl>=0.9' datasets accelerate"


class SFTFineTuningTask(TaskConfiguration):
    def __init__(
        self,
        model_name: str,
        dataset_name: str,
        env: Dict[str, str],
        new_model_name: Optional[str] = None,
        report_to: Optional[str] = None,
        per_device_train_batch_size: int = 4,
        per_device_eval_batch_size: int = 4,
        gradient_accumulation_steps: int = 1,
        learning_rate: float = 2e-4,
        max_grad_norm: float = 0.3,
        weight_decay: float = 0.001,
        lora_alpha: int = 16,
        lora_dropout: float = 0.1,
        lora_r: int = 64,
        max_seq_length: Optional[int] = None,
        use_4bit: bool = False,
        use_nested_quant: bool = True,
        bnb_4bit_compute_dtype: str = "bfloat16",
        bnb_4bit_quant_type: str = "nf4",
        num_train_epochs: float = 1,
        fp16: bool = False,
        bf16: bool = True,
        packing: bool = False,
        gradient_checkpointing: bool = True,
        optim: str = "adamw_torch_fused",
        lr_scheduler_type: str = "constant",
        max_steps: int = -1,
        warmup_ratio: float = 0.03,
        group_by_length: bool = True,
        save_steps: int = 0,
        logging_steps: int = 25,
        **task_kwargs,
    ):
        if "HF_TOKEN" not in env and "HUGGING_FACE_HUB_TOKEN" not in env:
            raise ValueError("env must carry HF_TOKEN (gated models, pushing the fine-tuned model)")
        if fp16 and bf16:
            raise ValueError("fp16 and bf16 are exclusive")
        args = dict(model_name=model_name, dataset_name=dataset_name, new_model_name=new_model_name,
                    report_to=report_to or "none", per_device_train_batch_size=per_device_train_batch_size,
                    per_device_eval_batch_size=per_device_eval_batch_size,
                    gradient_accumulation_steps=gradient_accumulation_steps, learning_rate=learning_rate,
                    max_grad_norm=max_grad_norm, weight_decay=weight_decay, lora_alpha=lora_alpha,
                    lora_dropout=lora_dropout, lora_r=lora_r, max_seq_length=max_seq_length, use_4bit=use_4bit,
                    use_nested_quant=use_nested_quant, bnb_4bit_compute_dtype=bnb_4bit_compute_dtype,
                    bnb_4bit_quant_type=bnb_4bit_quant_type, num_train_epochs=num_train_epochs, fp16=fp16,
                    bf16=bf16, packing=packing, gradient_checkpointing=gradient_checkpointing, optim=optim,
                    lr_scheduler_type=lr_scheduler_type, max_steps=max_steps, warmup_ratio=warmup_ratio,
                    group_by_length=group_by_length, save_steps=save_steps, logging_steps=logging_steps)
        flags = " ".join(f"--{k} {shlex.quote(str(v))}" for k, v in args.items() if v is not None)
        blob = base64.b64encode(_SCRIPT.read_bytes()).decode()
        commands = [
            _PIP + (" 'bitsandbytes>=0.45'" if use_4bit else ""),
            f"echo {blob} | base64 -d > {_SCRIPT_PATH}",
            # one process per GPU of the node (accelerate picks up every visible GPU); RCCL underneath
            f"accelerate launch --num_processes ${{DSTACK_GPUS_PER_NODE:-1}} {_SCRIPT_PATH} {flags}",
        ]
        env = {"PYTORCH_HIP_ALLOC_CONF": "expandable_segments:True", **env}
        super().__init__(type="task", commands=commands, env=env, **task_kwargs)
        object.__setattr__(self, "_sft_args", args)

    @property
    def sft_args(self) -> dict:
        return dict(self._sft_args)


__all__ = ["SFTFineTuningTask"]
