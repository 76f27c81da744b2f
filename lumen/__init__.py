"""lumen: MI355X-native LoRA fine-tuning and serving for Llama-class models."""
__version__ = "0.4.0"
