"""IE noise of the GPU path vs the float32 truth, next to the reference's own bf16 error (per question).

Run on the GPU box, once per kernel variant:  python tools/ie_noise_probe.py (variant knob: CRAM_PREFILL_VARIANT, read once at start)
"""
import gzip, json, os, sys
import numpy as np
sys.path.insert(0, '.')
from tests import tiny_models as tm
from tests.test_engine_cpu import ie_tolerance_check
from cram_amd.re_weighting import Find_Best_Heads
GOLD = 'tests/golden'
nq = json.load(gzip.open('data/nq_1000.json.gz', 'rt'))
root = '/tmp/tiny_probe'
for kind in ('qwen2', 'llama3'):
    obj = Find_Best_Heads(model_name=tm.save_model(kind, root))
    gold = [x for x in json.load(gzip.open(f'{GOLD}/tiny_ie.json.gz', 'rt')) if x['kind'] == kind and x['variant'] == 'fp32']
    truth = {x['idx']: x['ie'] for x in json.load(gzip.open(f'{GOLD}/tiny_ie_f32.json.gz', 'rt')) if x['kind'] == kind}
    for g in gold:
        rec = nq[g['idx']]
        ie = np.array(obj.cal_logits(question=rec['question'], paras=rec['ori_fake'] + rec['reranked_dense_ctxs'],
                                     scores=[0, 1, 1, 1, 1], wrong_answer=rec['wrong_answer']))
        t, r = np.array(truth[g['idx']]), np.array(g['ie'])
        print(os.environ.get('CRAM_PREFILL_VARIANT', '1'), kind, g['idx'], 'ie-err mean %.4f max %.4f | ref-err mean %.4f max %.4f' % (
            np.abs(ie - t).mean(), np.abs(ie - t).max(), np.abs(r - t).mean(), np.abs(r - t).max()))
