"""profiles/pmc_traffic.json for bench.py's roofline "traffic": HBM bytes per launch of each bench
timer (kernel group) summed over its kernels, from a bench_tools/pmc_summary.py output.

    python bench_tools/pmc_to_traffic.py gpurun_out/<tag>/summary.json > profiles/pmc_traffic.json
"""
import json
import sys

GROUPS = {
    "k_decode": ["k_decode_sig", "k_pk_gather"],
    "k_subgroup": ["k_subgroup"],
    "k_msm_g2": ["void k_msm_bucket<ssb::fp2>", "void k_msm_window<ssb::fp2>"],
    "k_msm_g1": ["void k_msm_bucket<ssb::fp>", "void k_msm_window_seq<ssb::fp>", "k_msm_horner"],
    "k_rlc_pk": ["k_rlc_pk"],
    "k_miller": ["k_miller_pairs"],
    "k_final": ["k_fp12_prod8", "k_final_lane"],
    "k_hash_to_g2": ["k_h2c_u", "k_h2c_map", "k_h2c_clear", "k_h2c_affine"],
    "k_combine_fast": ["k_combine_fast"],
}


def main(path):
    d = json.load(open(path))
    out = {"_doc": "HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024), rocprofv3 --pmc in separate "
                   "passes (bench_tools/pmc.sh, depth-1 bench run), summed over each timer's kernels"}
    for g, ks in GROUPS.items():
        vals = [d[k]["hbm_bytes_per_launch"] for k in ks if k in d and "hbm_bytes_per_launch" in d[k]]
        if vals:
            out[g] = {"hbm_bytes_per_launch": sum(vals), "kernels": ks}
    json.dump(out, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1])
