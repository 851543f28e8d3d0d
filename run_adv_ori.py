"""Drop-in for the reference's run_adv_ori.py (APR / BPR-MF on the MI355X path).

    python run_adv_ori.py --model apr --dataset Video --epochs 2000 --adv_epoch 1000 \
        --verbose 20 --eval_mode all --embed_size 64
"""
import importlib
import sys

if __name__ == "__main__":
    sys.exit(importlib.import_module("adversarial-collaborative-filtering_amd.cli").main(sys.argv[1:], "ori"))
