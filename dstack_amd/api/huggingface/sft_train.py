"""Supervised fine-tuning with LoRA (optionally on a 4-bit base) for ``SFTFineTuningTask``.

This file is shipped INTO the task's container (base64 in the task's commands) and runs there with
transformers + peft + trl + datasets installed by the task.  On MI355X (288 GB HBM3E) a bf16 base of
up to ~70B parameters fits on one GPU, so ``--use_4bit`` is off unless asked for; when it is on,
bitsandbytes' ROCm backend quantises the base.  Multi-GPU runs go through ``accelerate launch``
(one process per GPU, RCCL).
"""

import argparse
import os


def _bool(v: str) -> bool:
    return str(v).lower() in ("1", "true", "yes", "on")


def parse_args(argv=None):
    p = argparse.ArgumentParser("dstack-sft")
    p.add_argument("--model_name", required=True)
    p.add_argument("--dataset_name", required=True)
    p.add_argument("--new_model_name", default=None)
    p.add_argument("--report_to", default="none")
    p.add_argument("--per_device_train_batch_size", type=int, default=4)
    p.add_argument("--per_device_eval_batch_size", type=int, default=4)
    p.add_argument("--gradient_accumulation_steps", type=int, default=1)
    p.add_argument("--learning_rate", type=float, default=2e-4)
    p.add_argument("--max_grad_norm", type=float, default=0.3)
    p.add_argument("--weight_decay", type=float, default=0.001)
    p.add_argument("--lora_alpha", type=int, default=16)
    p.add_argument("--lora_dropout", type=float, default=0.1)
    p.add_argument("--lora_r", type=int, default=64)
    p.add_argument("--max_seq_length", type=int, default=None)
    p.add_argument("--use_4bit", type=_bool, default=False)
    p.add_argument("--use_nested_quant", type=_bool, default=True)
    p.add_argument("--bnb_4bit_compute_dtype", default="bfloat16")
    p.add_argument("--bnb_4bit_quant_type", default="nf4")
    p.add_argument("--num_train_epochs", type=float, default=1)
    p.add_argument("--fp16", type=_bool, default=False)
    p.add_argument("--bf16", type=_bool, default=True)
    p.add_argument("--packing", type=_bool, default=False)
    p.add_argument("--gradient_checkpointing", type=_bool, default=True)
    p.add_argument("--optim", default="adamw_torch_fused")
    p.add_argument("--lr_scheduler_type", default="constant")
    p.add_argument("--max_steps", type=int, default=-1)
    p.add_argument("--warmup_ratio", type=float, default=0.03)
    p.add_argument("--group_by_length", type=_bool, default=True)
    p.add_argument("--save_steps", type=int, default=0)
    p.add_argument("--logging_steps", type=int, default=25)
    p.add_argument("--output_dir", default="./results")
    return p.parse_args(argv)


def main(argv=None):
    a = parse_args(argv)
    import torch
    from datasets import load_dataset
    from peft import LoraConfig
    from transformers import AutoModelForCausalLM, AutoTokenizer
    from trl import SFTTrainer

    quant = None
    if a.use_4bit:
        from transformers import BitsAndBytesConfig

        quant = BitsAndBytesConfig(load_in_4bit=True, bnb_4bit_quant_type=a.bnb_4bit_quant_type,
                                   bnb_4bit_compute_dtype=getattr(torch, a.bnb_4bit_compute_dtype),
                                   bnb_4bit_use_double_quant=a.use_nested_quant)
    dtype = torch.bfloat16 if a.bf16 else (torch.float16 if a.fp16 else torch.float32)
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    model = AutoModelForCausalLM.from_pretrained(a.model_name, quantization_config=quant, torch_dtype=dtype,
                                                 device_map={"": local_rank})
    model.config.use_cache = False
    tok = AutoTokenizer.from_pretrained(a.model_name, trust_remote_code=True)
    if tok.pad_token is None:
        tok.pad_token = tok.eos_token
    tok.padding_side = "right"
    data = load_dataset(a.dataset_name, split="train")
    lora = LoraConfig(lora_alpha=a.lora_alpha, lora_dropout=a.lora_dropout, r=a.lora_r, bias="none",
                      task_type="CAUSAL_LM")
    common = dict(output_dir=a.output_dir, num_train_epochs=a.num_train_epochs,
                  per_device_train_batch_size=a.per_device_train_batch_size,
                  per_device_eval_batch_size=a.per_device_eval_batch_size,
                  gradient_accumulation_steps=a.gradient_accumulation_steps, optim=a.optim,
                  save_steps=a.save_steps, logging_steps=a.logging_steps, learning_rate=a.learning_rate,
                  weight_decay=a.weight_decay, fp16=a.fp16, bf16=a.bf16, max_grad_norm=a.max_grad_norm,
                  max_steps=a.max_steps, warmup_ratio=a.warmup_ratio, group_by_length=a.group_by_length,
                  lr_scheduler_type=a.lr_scheduler_type, report_to=a.report_to,
                  gradient_checkpointing=a.gradient_checkpointing)
    try:  # trl >= 0.9: SFT options live on SFTConfig
        from trl import SFTConfig

        args = SFTConfig(**common, packing=a.packing, dataset_text_field="text",
                         **({"max_seq_length": a.max_seq_length} if a.max_seq_length else {}))
        trainer = SFTTrainer(model=model, train_dataset=data, peft_config=lora, args=args)
    except ImportError:
        from transformers import TrainingArguments

        trainer = SFTTrainer(model=model, train_dataset=data, peft_config=lora, dataset_text_field="text",
                             max_seq_length=a.max_seq_length, tokenizer=tok, args=TrainingArguments(**common),
                             packing=a.packing)
    trainer.train()
    if a.new_model_name:
        trainer.model.save_pretrained(a.new_model_name)
        tok.save_pretrained(a.new_model_name)
        if os.environ.get("HF_TOKEN") and local_rank == 0:
            trainer.model.push_to_hub(a.new_model_name)
            tok.push_to_hub(a.new_model_name)


if __name__ == "__main__":
    main()
