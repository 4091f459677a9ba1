#!/usr/bin/env python3
"""Summarise a parity log (one JSON line per tests/hip_util.assert_close check,
written when SRCNN_PARITY_LOG is set during `pytest -m gpu`):

    SRCNN_PARITY_LOG=gpurun_out/parity.jsonl python -m pytest tests -m gpu
    python tools/parity_summary.py gpurun_out/parity.jsonl > profiles/<round>_parity/summary.json

Fields: check count, checks against the exact (double-precision) result,
the largest normwise error, the largest elementwise relative error on
significant elements, how many checks stay within 1e-4 elementwise, and the
ten checks with the largest elementwise error.
"""
import json
import sys


def main(path):
    recs = [json.loads(l) for l in open(path) if l.strip()]
    exact = [r for r in recs if r.get("elementwise") is not None]
    out = {
        "checks": len(recs),
        "with_exact_reference": len(exact),
        "max_normwise": max((r["normwise"] for r in recs), default=None),
        "max_elementwise_no_floor": max((r["elementwise"] for r in exact if not r.get("abs_floor")), default=None),
        "elementwise_within_1e-4": sum(1 for r in exact if r["elementwise"] <= 1e-4),
        "elementwise_beyond_own_bound": sum(1 for r in exact if r.get("n_over")),
        "worst": sorted(({k: r[k] for k in ("what", "n", "normwise", "elementwise", "elementwise_fp32_oracle",
                                            "abs_floor") if k in r} for r in exact),
                        key=lambda r: -r["elementwise"])[:10],
    }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
