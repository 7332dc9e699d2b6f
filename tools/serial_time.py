import sys, os, time
sys.path.insert(0,'tests'); sys.path.insert(0,'.')
import torch; torch.cuda.init()
import oracle_lib as ol, parity_util as pu
golden='tests/golden'
iset, env, cfg = pu.load_env(golden, "instset-classic.cfg", seed=5)
n=cfg.world_x*cfg.world_y
g=ol.Backend("gpu", cfg, iset, env, ncells=n)
g.set_orgs(0, pu.pop_genomes(golden, iset)[:n], deterministic=False)
t=time.time()
for u in range(5):
    s=g.run_serial_update()
print("serial gpu s/update", (time.time()-t)/5, s.num_organisms, s.insts_executed)
