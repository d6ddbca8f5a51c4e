"""nanoGPT-compatible sampling entry point: ``python sample.py --out_dir=... --start=...``."""
from nanosandbox_amd.sample import main

if __name__ == "__main__":
    main()
