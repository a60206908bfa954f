"""Fold the two halves of tools/cfg5_share.py (--tiles 0:8 and 8:16) into one phase summary.

    python tools/cfg5_summary.py share_a.json share_b.json out.json"""
import json
import sys


def main(pa_path, pb_path, out_path):
    a, b = json.load(open(pa_path)), json.load(open(pb_path))
    pa, pb = a["phases_s"], b["phases_s"]
    tiles = a["per_tile"] + b["per_tile"]
    rep = sum(t["replay_grids_s"] for t in tiles)
    comb = sum(t["combine_s"] for t in tiles)
    setup = (pa["setup_s"] + pb["setup_s"]) / 2
    chains = (pa["chains_s"] + pb["chains_s"]) / 2
    pg = (pa["param_grids_s"] + pb["param_grids_s"]) / 2
    sites = sum(t["sites"] for t in tiles)
    out = {"workload": a["workload"],
           "measured_in": "two processes (tools/cfg5_share.py --tiles 0:8 and 8:16; gpurun's 20-minute command "
                          "limit): each repeats the same deterministic fit, the per-tile replays add",
           "phases_s": {"setup_partition_glm_subsets": setup, "chains_5000_iterations": chains, "parameter_grids": pg,
                        "kriging_replay_and_grids_16_tiles": rep, "combine_shard_mean_16_tiles": comb,
                        "total_excluding_data_generation": setup + chains + pg + rep + comb},
           "chains_s_per_process": [pa["chains_s"], pb["chains_s"]],
           "test_sites": sites, "kept_states": 1251, "subsets": 32,
           "x_refreshes_per_kept_sample": a["x_refreshes_per_kept_sample"],
           "draws": 32 * sites * 1251, "draws_per_s_over_replay": 32 * sites * 1251 / rep,
           "per_tile_replay_s": [round(t["replay_grids_s"], 2) for t in tiles]}
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps(out["phases_s"]), out["draws_per_s_over_replay"] / 1e6)


if __name__ == "__main__":
    main(*sys.argv[1:4])
