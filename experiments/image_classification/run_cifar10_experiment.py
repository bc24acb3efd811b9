#!/usr/bin/env python3
"""Image classification under attack (README.md:101-102 of the reference; missing there).

ResNet-32 on CIFAR-10-shaped data, 2 pipeline stages, gradient + data poisoning on stage 1 from
epoch 2; writes the experiment artefacts (JSON / CSV / PNG / Markdown) under results/.
Extra flags are forwarded to the experiment runner (e.g. --device cuda:0 --nodes 4)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from trustworthy_dl.experiments.runner import main  # noqa: E402

if __name__ == "__main__":
    main(["--model", "resnet32", "--dataset", "cifar10", "--nodes", "2", "--epochs", "4", "--attack",
          "--batch-size", "64", "--lr", "1e-3", "--batches-per-epoch", "20"] + sys.argv[1:])
