"""Drop-in for the reference's run_adv.py (flag surface of run_adv.py:15-54)."""
import importlib
import sys

if __name__ == "__main__":
    sys.exit(importlib.import_module("adversarial-collaborative-filtering_amd.cli").main(sys.argv[1:], "adv"))
