#!/usr/bin/env python3
"""configs[0]'s stage wall alone (bench.pipeline_stage_wall): the fixed and ideal 3-tap stages over
the 7 golden images through the host API, fresh and overwrite runs, with their breakdowns.
Optional arguments: writer-thread counts to compare (FIR_STAGE_WRITERS), e.g. 4 8 16."""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402

res = {}
for w in sys.argv[1:] or [os.environ.get("FIR_STAGE_WRITERS", "8")]:
    os.environ["FIR_STAGE_WRITERS"] = str(w)
    res[f"writers_{w}"] = bench.pipeline_stage_wall()
print(json.dumps(res, indent=1))
