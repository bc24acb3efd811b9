#!/usr/bin/env python3
"""Language modelling with model poisoning (README.md:104-105 of the reference; missing there).

GPT-2 (configs/gpt2_distributed.yaml schema) over 4 pipeline stages with the attacker poisoning
gradients of the targeted stages; writes the experiment artefacts under results/.
Extra flags are forwarded to the experiment runner (e.g. --config configs/gpt2_distributed.yaml)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from trustworthy_dl.experiments.runner import main  # noqa: E402

if __name__ == "__main__":
    main(["--model", "gpt2-small", "--dataset", "openwebtext", "--nodes", "4", "--epochs", "4", "--attack",
          "--batch-size", "8", "--seq-len", "128", "--batches-per-epoch", "20"] + sys.argv[1:])
