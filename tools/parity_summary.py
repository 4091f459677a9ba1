#!/usr/bin/env python3
"""Summarise a parity log (one JSON line per tests/hip_util.assert_close check,
written when SRCNN_PARITY_LOG is set during `pytest -m gpu`):

    SRCNN_PARITY_LOG=gpurun_out/parity.jsonl python -m pytest tests -m gpu
    python tools/parity_summary.py gpurun_out/parity.jsonl > profiles/<round>_parity/summary.json

Fields: check count, checks against the exact (double-precision) result,
the largest normwise error, the largest elementwise relative error on
significant elements, how many checks stay within 1e-4 elementwise, and the
ten checks with the largest elementwise error.  The masked-parity tests
(tests/test_parity_masks_gpu.py) add two kinds of record: ReLU-decision flip
counts per layer (`flips_A*`, `ambiguous_A*`) and checks whose elements past
the relative tolerance are judged against the fp32 rounding bound
(`n_over_rtol`, `rounding_ratio_max`); both are summarised separately.
"""
import json
import sys


def main(path):
    allrecs = [json.loads(l) for l in open(path) if l.strip()]
    flips = [r for r in allrecs if "flips_A1" in r]
    recs = [r for r in allrecs if "normwise" in r]
    bounded = [r for r in recs if "rounding_ratio_max" in r]
    exact = [r for r in recs if r.get("elementwise") is not None]
    out = {
        "checks": len(recs),
        "with_exact_reference": len(exact),
        "max_normwise": max((r["normwise"] for r in recs), default=None),
        "max_elementwise_no_floor": max((r["elementwise"] for r in exact if not r.get("abs_floor")), default=None),
        "elementwise_within_1e-4": sum(1 for r in exact if r["elementwise"] <= 1e-4),
        "elementwise_beyond_own_bound": sum(1 for r in exact if r.get("n_over")),
        "rounding_clause_checks": len(bounded),
        "rounding_clause_elements_past_rtol": sum(r["n_over_rtol"] for r in bounded),
        "rounding_ratio_max": max((r["rounding_ratio_max"] for r in bounded), default=None),
        "rounding_clause_scale": "0.25 x the probabilistic estimate u sqrt(n) sum|terms| (hip_util.K_ROUND)",
        "rounding_only_elements": sum(r.get("n_round_only", 0) for r in bounded),
        "flip_records": len(flips),
        "flips_total": {k: sum(r[k] for r in flips) for k in ("flips_A1", "flips_A2", "flips_A3")},
        "ambiguous_total": {k: sum(r[k] for r in flips) for k in ("ambiguous_A1", "ambiguous_A2", "ambiguous_A3")},
        "worst": sorted(({k: r[k] for k in ("what", "n", "normwise", "elementwise", "elementwise_fp32_oracle",
                                            "abs_floor") if k in r} for r in exact),
                        key=lambda r: -r["elementwise"])[:10],
    }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
