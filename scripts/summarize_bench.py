"""Print the key numbers of a bench.py JSON line (usage: python scripts/summarize_bench.py FILE)."""
import json
import sys

b = json.loads([l for l in open(sys.argv[1]) if l.strip().startswith("{")][-1])
r = b.get("roofline_fwd", b["roofline"])
rb = b.get("roofline_back")
print(f"headline {b['value']:.1f} {b['unit']} ({b['ms_per_step']:.3f} ms/step, {b['config']['nodes']} nodes, "
      f"{b['n_gpus']} GPU)  fwd {r['avg_launch_ms'] * 1e3:.2f} us (b2b {r['avg_launch_ms_back_to_back'] * 1e3:.2f}) "
      f"frac {r['frac']}  lds {r['lds']['frac']:.3f}"
      + (f"  back {rb['avg_launch_ms'] * 1e3:.2f} us frac {rb['frac']} lds {rb['lds']['frac']:.3f}" if rb else ""))
if "cpu_baseline" in b:
    c = b["cpu_baseline"]
    print(f"cpu {c['value']:.2f} {c['unit']} on {c['cores']} cores, rel_fro {c['rel_fro']:.2e}")
if "weak8" in b:
    print(f"weak8 {b['weak8']['value']:.1f} ({b['weak8']['ms_per_step']:.3f} ms/step)")
for s in b.get("strong", []):
    print(f"strong {s['config']} {s['value']:.1f} ({s['ms_per_step']:.2f} ms/step)")
for k, p in sorted(b.get("proxy_8gpu", {}).items()):
    if not isinstance(p, dict):
        continue
    if "T1_ms_per_step" not in p:  # weak8@8: the N = 8 weak headline itself
        print(f"proxy {k}: {p['nodes']} nodes on {p['ranks']} ranks, predicted {p['predicted_value']:.0f} "
              f"node-updates/s ({p['predicted_ms_per_step']:.2f} ms/step), {p['predicted_speedup']:.2f}x the "
              f"one-GPU headline (one link {p['predicted_speedup_one_link']:.2f}x)")
        continue
    sh = " | ".join(f"r{s['rank']}: V={s['local_nodes']} vb={s['vb']} H={s['halo_rows']} E={s['stored_edges']} "
                    f"{s['ms_per_step']:.2f} ms (cons {s.get('consensus_ms', float('nan')):.2f}) + ex "
                    f"{s['exchange'].get('ms_conservative', s['exchange']['ms_direct']):.2f} ({s['exchange']['mode']}) "
                    f"z {s.get('z', '?')}"
                    for s in p["shares"])
    print(f"proxy {k}: T1 {p['T1_ms_per_step']:.2f} ms, per-node ratio {p['per_node_cost_ratio']:.3f}, "
          f"speedup {p['predicted_speedup']:.2f}x (one link {p['predicted_speedup_one_link']:.2f}x, direct "
          f"{p.get('predicted_speedup_direct', float('nan')):.2f}x)  [{sh}]")
