"""QLoRA with TRL: the base model is loaded in 4-bit NF4 (bitsandbytes), LoRA adapters on every
linear projection train in bf16, gradient checkpointing keeps activations small."""
import argparse

import torch
from datasets import load_dataset
from peft import LoraConfig
from transformers import AutoModelForCausalLM, AutoTokenizer, BitsAndBytesConfig
from trl import SFTConfig, SFTTrainer


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", required=True)
    ap.add_argument("--dataset", required=True)
    ap.add_argument("--output", required=True)
    ap.add_argument("--max-steps", type=int, default=1000)
    a = ap.parse_args()
    quant = BitsAndBytesConfig(load_in_4bit=True, bnb_4bit_quant_type="nf4", bnb_4bit_use_double_quant=True,
                               bnb_4bit_compute_dtype=torch.bfloat16)
    model = AutoModelForCausalLM.from_pretrained(a.model, quantization_config=quant, torch_dtype=torch.bfloat16,
                                                 device_map={"": 0})
    tok = AutoTokenizer.from_pretrained(a.model)
    tok.pad_token = tok.pad_token or tok.eos_token
    lora = LoraConfig(r=16, lora_alpha=32, lora_dropout=0.05, task_type="CAUSAL_LM",
                      target_modules=["q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj"])
    cfg = SFTConfig(output_dir=a.output, max_steps=a.max_steps, per_device_train_batch_size=8,
                    gradient_accumulation_steps=2, learning_rate=2e-4, bf16=True, logging_steps=10,
                    gradient_checkpointing=True, save_steps=200, dataset_text_field="text", max_seq_length=2048)
    trainer = SFTTrainer(model=model, args=cfg, train_dataset=load_dataset(a.dataset, split="train"),
                         peft_config=lora, processing_class=tok)
    trainer.train()
    trainer.save_model(a.output)


if __name__ == "__main__":
    main()
