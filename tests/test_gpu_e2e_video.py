"""End-to-end statistical anchor on the reference's own Video data (HR@10 within
±0.002 of the published run: north_star's end-to-end bar, checked on the one
published APR run whose train file ships with the reference).

Protocol of out/janEval/Video_apr_d64_e0.500000_l1.000000_2020_01_24_12_07_42.out
(run_adv_ori.py --model apr --dataset Video --epochs 2000 --adv_epoch 1000
--verbose 20 --eval_mode all --embed_size 64) through this build's CLI; ~20 s on
one MI355X.  Anchors (tests/golden/published_logs.json, parsed from that log):
  best-epoch K=10 row: HR 0.0650, NDCG 0.0331   (log lines 105, 115)
  |P|, |Q| at the BPR->APR switch (epoch 1000): 619.33, 562.31   (line 54)
  |P|, |Q| at epoch 2000: 850.34, 828.95                           (line 102)
The run is bit-reproducible (deterministic kernels, seeded device sampler), so
the test is deterministic; the sampler stream itself differs from the
reference's (its forked Pool workers share one numpy RNG state).
"""
import json
import os
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "Video_apr_d64_e0.500000_l1.000000_2020_01_24_12_07_42.out"


def test_video_apr_hr10_within_0002_of_published():
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import e2e_video
    summary, text = e2e_video.run(epochs=2000, adv_epoch=1000, verbose=20, model="apr", seed=0, out=None)
    assert summary["rc"] in (0, None)
    ref = json.load(open(os.path.join(REPO, "tests", "golden", "published_logs.json")))[REF]
    _, hr_ref, ndcg_ref, _ = ref["best"][9]
    assert abs(summary["hr10"] - hr_ref) <= 0.002, summary
    assert abs(summary["ndcg10"] - ndcg_ref) <= 0.002, summary
    ours = e2e_video.trajectory(text)
    theirs = {e["epoch"]: (e["normP"], e["normQ"]) for e in ref["epochs"]}
    for ep in (1000, 2000):
        for k, name in ((0, "|P|"), (1, "|Q|")):
            got, want = ours[ep][2 + k], theirs[ep][k]
            assert abs(got - want) <= 0.02 * want, f"epoch {ep} {name}: {got} vs published {want}"
