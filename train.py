"""nanoGPT-compatible entry point: ``python train.py config/x.py --key=value``.

Runs the MI355X-native trainer (``nanosandbox_amd.train``); see that module
for what is contract (nanoGPT) and what is redesigned for gfx950.
"""
from nanosandbox_amd.train import main

if __name__ == "__main__":
    main()
