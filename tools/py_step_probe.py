import sys, time, os
sys.path[:0]=['.','mpas-model_amd']
from mpas_dycore import Dycore
from mpas_dycore.cases import jw_case
c=jw_case(163842,K=56,ns=1,order=3); dt=float(c['dt'])
for summ in (1, 0):
    dy=Dycore(c,device=0); dy.init_diagnostics(dt); dy.use_graph(True)
    dy.lib.mpas_dyc_set_summary(dy.h, summ)
    for it in range(2): dy.atm_timestep(dt,it+1); dy.shift_time_levels()
    dy.synchronize(); t0=time.perf_counter()
    for it in range(2,10): dy.atm_timestep(dt,it+1); dy.shift_time_levels()
    dy.synchronize(); print('summary',summ,'ms/dt',(time.perf_counter()-t0)/8*1e3, flush=True)
    dy.close()
