from .gpt import GPT, GPTConfig, MI355X_BF16_PEAK_FLOPS  # noqa: F401
