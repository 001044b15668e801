import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from emqx_amd import Context
from emqx_amd.engine import gen_filter_codes, render_codes
ctx = Context(0)
codes = gen_filter_codes(1, 10_000_000)
idx = ctx.build_index(render_codes(codes))
db, do, _ = ctx.gen_topics_device(codes, 1, 0, 10_000_000)
r = ctx.match_device(idx, db, do, 10_000_000); ctx.synchronize(); r.free()
