"""Drop-in for the reference's run.py (flag surface of run.py:25-75; models bpr,
apr, bpr-tf, neumf, aneumf on the MI355X path)."""
import importlib
import sys

if __name__ == "__main__":
    importlib.import_module("adversarial-collaborative-filtering_amd.run_cli").main(sys.argv[1:])
