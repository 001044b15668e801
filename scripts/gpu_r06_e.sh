#!/bin/bash
# Round 6, GPU call e: the C5
# bench line on the new library: kernel, update (observed mirror loads), the
# multi-device block (two replicas on this GPU: replication, host batch spread,
# replicated updates) and the host link.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_e
mkdir -p $O
summ() {
python3 - "$1" <<'PY'
import json, sys
d=json.load(open(sys.argv[1]))
r=d['roofline']; de=d['detail']
print(sys.argv[1], round(d['value']/1e9,3),'G/s', round(d['ms_per_step'],3),'ms/step kernel', round(r['kernel_ms'],3), 'frac', round(r['frac'],3), 'src', de.get('index_source'), 'dev GB', round(de['index_device_bytes']/1e9,2))
print(' import', json.dumps({k: v for k, v in de.items() if k.startswith('index_import')}))
print(' host_io', round(de.get('host_io_topics_per_s',0)/1e9,3), 'link frac', round(de.get('host_io_link',{}).get('h2d_frac_of_peak',0),3))
u=de.get('index_update',{}); print(' update', round(u.get('update_ms',0),3), 'first', round(u.get('first_update_ms',0),2), 'mirror', u.get('first_includes_mirror_download'), u.get('first_mirror_bytes'))
m=de.get('multi_device',{}); ur=m.get('index_update_replicas',{})
print(' multi', m.get('devices'), 'replicate_ms', round(m.get('replicate_ms',0),2), 'host_io_multi', round(m.get('host_io_multi_topics_per_s',0)/1e9,3), 'upd_rep', round(ur.get('update_ms',0),3), 'vs single', round(ur.get('vs_single_device',0),3), [ (round(x['ms'],2), x['kind'], x['replica_mode'], x['mirror_loaded']) for x in ur.get('rounds',[])])
print(' parity', d.get('parity_sample',{}).get('ok'))
PY
}
timeout -k 10 1000 python3 -u bench.py --config c5 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
tail -n 1 $O/bench_c5.log > $O/bench_c5.json && summ $O/bench_c5.json
