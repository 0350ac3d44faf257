#!/bin/bash
# rocprofv3 kernel stats of the C2 line alone (acoustic model, B = 32, T_mel = 512)
set -o pipefail
OUT=gpurun_out/c2prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python bench.py --mode c2 --steps 10 --cpu-seconds 0 > $OUT/bench.out 2>&1 || { tail -20 $OUT/bench.out; exit 1; }
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/c2prof/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total ms", tot / 1e6)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    print(f'{float(r["TotalDurationNs"])/1e6:8.2f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:150]}')


def cls(n):  # kernel class of the C2 breakdown
    if "layernorm" in n or "ln_" in n:
        return "LayerNorm (+ residual, pad-row zeroing)"
    if "attn" in n or "attention" in n:
        return "attention"
    if "conv_splitk_reduce" in n or "conv1d_kernel<float, float, float" in n:
        return "fp32 short-sequence convs (encoder / predictors, T_src = 12; split reduction)"
    if "conv1d_kernel<" in n:  # template <input, compute, output, ...>: bf16 compute
        return "bf16-compute convs over T_mel (decoder FFN w_1 / w_2, q/k/v, fc; PostNet; mel_linear)"
    return "glue (embeddings, VFE, length regulator, heads, masks, casts)"


agg = {}
for r in rows:
    c = cls(r["Name"])
    a = agg.setdefault(c, [0.0, 0])
    a[0] += float(r["TotalDurationNs"])
    a[1] += int(r["Calls"])
print("\nper kernel class (trace totals over all bench launches; share of kernel time):")
for c, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
    print(f"{t / tot * 100:6.1f} %  {t / 1e6:8.2f} ms  {n:6d} launches  {c}")
PY
rm -f $OUT/run_kernel_trace.csv
