"""Scaling analysis over the metrics CSV (reference scripts/compare_training.py:16-168).

Same quantities as the reference -- speedup = baseline_time / time and
efficiency % = speedup / num_gpus * 100 (:46-47), a console table (:52-69), findings (:72-101)
and a 2x2 figure of time / speedup / memory / efficiency-vs-ideal saved at dpi 300 (:104-168) --
plus the token-throughput view lumen records (``tokens_per_second``), which is the headline
metric and does not depend on how many samples each run was given.  The baseline row is the
``baseline`` experiment when present, else the 1-GPU row of each strategy.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import pandas as pd


def load_and_calculate(csv_path: str = "results/training_metrics.csv") -> pd.DataFrame:
    df = pd.read_csv(csv_path)
    if df.empty:
        return df
    # keep the latest row per experiment (re-runs append)
    df = df.groupby("experiment", as_index=False, sort=False).last()
    for c in ("num_gpus", "training_time_hours", "samples_per_second", "peak_memory_gb",
              "final_loss", "tokens_per_second", "tflops_per_gpu"):
        if c in df:
            df[c] = pd.to_numeric(df[c], errors="coerce")
    base = df[df["experiment"] == "baseline"]
    speed, eff, tok_speed, tok_eff = [], [], [], []
    for _, r in df.iterrows():
        ref = base if len(base) else df[(df["strategy"] == r["strategy"]) & (df["num_gpus"] == 1)]
        if len(ref) and r["training_time_hours"] > 0:
            s = float(ref["training_time_hours"].iloc[0]) / float(r["training_time_hours"])
        else:
            s = float("nan")
        speed.append(s)
        eff.append(s / r["num_gpus"] * 100.0)
        if "tokens_per_second" in df and len(ref) and ref["tokens_per_second"].iloc[0] > 0:
            ts = float(r["tokens_per_second"]) / float(ref["tokens_per_second"].iloc[0])
        else:
            ts = float("nan")
        tok_speed.append(ts)
        tok_eff.append(ts / r["num_gpus"] * 100.0)
    df["speedup"] = speed
    df["efficiency"] = eff
    df["token_speedup"] = tok_speed
    df["token_efficiency"] = tok_eff
    return df.sort_values(["zero_stage", "num_gpus"]).reset_index(drop=True)


def format_table(df: pd.DataFrame) -> str:
    cols = ["experiment", "num_gpus", "zero_stage", "training_time_hours", "samples_per_second",
            "peak_memory_gb", "final_loss", "speedup", "efficiency"]
    cols += [c for c in ("tokens_per_second", "token_speedup", "token_efficiency") if c in df]
    return df[[c for c in cols if c in df]].to_string(index=False, float_format=lambda v: f"{v:.3f}")


def findings(df: pd.DataFrame) -> List[str]:
    out = []
    if df.empty:
        return out
    fastest = df.loc[df["training_time_hours"].idxmin()]
    out.append(f"Fastest run: {fastest['experiment']} ({fastest['training_time_hours']:.3f} h)")
    multi = df[df["num_gpus"] > 1]
    if len(multi):
        best = multi.loc[multi["efficiency"].idxmax()]
        out.append(f"Best multi-GPU scaling efficiency: {best['experiment']} "
                   f"({best['efficiency']:.1f}%)")
    lean = df.loc[df["peak_memory_gb"].idxmin()]
    out.append(f"Lowest peak memory per GPU: {lean['experiment']} ({lean['peak_memory_gb']:.2f} GB)")
    if "tokens_per_second" in df and df["tokens_per_second"].notna().any():
        top = df.loc[df["tokens_per_second"].idxmax()]
        out.append(f"Highest token throughput: {top['experiment']} "
                   f"({top['tokens_per_second']:.0f} tok/s)")
    return out


def plot(df: pd.DataFrame, out_path: str = "results/plots/training_comparison.png") -> Optional[str]:
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        return None
    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    fig, ax = plt.subplots(2, 2, figsize=(14, 10))
    for stage, g in df.groupby("zero_stage"):
        lbl = "baseline" if stage == 0 else f"ZeRO-{stage}"
        g = g.sort_values("num_gpus")
        ax[0, 0].plot(g["num_gpus"], g["training_time_hours"], "o-", label=lbl)
        ax[0, 1].plot(g["num_gpus"], g["speedup"], "o-", label=lbl)
        ax[1, 0].bar([f"{lbl}\n{n}gpu" for n in g["num_gpus"]], g["peak_memory_gb"], label=lbl)
        ax[1, 1].plot(g["num_gpus"], g["efficiency"], "o-", label=lbl)
    n = sorted(df["num_gpus"].unique())
    ax[0, 1].plot(n, n, "k--", label="ideal")
    ax[1, 1].axhline(100.0, color="k", ls="--", label="ideal")
    titles = [("Training time", "hours"), ("Speedup vs baseline", "x"),
              ("Peak memory per GPU", "GB"), ("Scaling efficiency", "%")]
    for a, (t, y) in zip(ax.flat, titles):
        a.set_title(t)
        a.set_ylabel(y)
        a.legend()
        a.grid(alpha=0.3)
    for a in (ax[0, 0], ax[0, 1], ax[1, 1]):
        a.set_xlabel("GPUs")
    fig.tight_layout()
    fig.savefig(out_path, dpi=300)
    plt.close(fig)
    return out_path


def compare(csv_path: str = "results/training_metrics.csv",
            plot_path: str = "results/plots/training_comparison.png") -> Dict:
    df = load_and_calculate(csv_path)
    print("=" * 90)
    print("TRAINING SCALING COMPARISON")
    print("=" * 90)
    print(format_table(df))
    print()
    for f in findings(df):
        print(" *", f)
    p = plot(df, plot_path) if len(df) else None
    if p:
        print(f"\nPlot saved to {p}")
    return {"table": df, "plot": p}
