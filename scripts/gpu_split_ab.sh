cd "${GRAFT_REPO_ROOT}"; O=gpurun_out/split; mkdir -p $O
ZB_SPLIT=1 timeout -k 10 90 python -c "
import torch; from zbot_lab_amd.sim import ZbotSim; from zbot_lab_amd import model as zm
s=ZbotSim(64, zm.TaskCfg(), seed=1); s.reset()
for _ in range(5): o,r,t,u=s.step(torch.randn(64,6,device='cuda'))
torch.cuda.synchronize(); print('tiny split ok', float(r.sum()))
" > $O/tiny.log 2>&1 || { cat $O/tiny.log; exit 1; }
tail -1 $O/tiny.log
for v in 0 1; do ZB_SPLIT=$v N=4096 STEPS=200 timeout -k 10 200 python scripts/bitident.py > $O/bit$v.log 2>&1 || { tail -5 $O/bit$v.log; exit 1; }; grep walking $O/bit$v.log; done
for r in 1 2; do for v in 0 1; do
  ZB_SPLIT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]);print('split=$v value %.4e ms/step %.4f kernel_ms %.4f'%(d['value'],d['ms_per_step'],d['roofline']['kernel_ms']))" | tee -a $O/summary.txt
done; done
