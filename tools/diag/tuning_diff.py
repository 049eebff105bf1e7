"""Print, as one JSON object, the entries of a scratch tuning table that differ from ops/gemv_tuning.json (for
NLS_TUNING_EXTRA A/Bs of a fresh tuner run before it is merged): python tools/diag/tuning_diff.py <scratch.json>"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
cur = json.load(open(os.path.join(ROOT, "nats_llm_studio_amd", "ops", "gemv_tuning.json")))
new = json.load(open(sys.argv[1]))
print(json.dumps({k: v for k, v in new.items() if cur.get(k) != v}))
