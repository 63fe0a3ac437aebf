cd $GRAFT_REPO_ROOT
for n in 64 4096; do
timeout -k 10 200 python bench.py --steps 1000 --warmup 50 --no-cpu-baseline --envs-per-gpu $n | python -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print('n=$n %.4e ms %.4f k %.4f'%(d['value'],d['ms_per_step'],d['roofline']['kernel_ms']))" || exit 1
done
timeout -k 10 200 python -c "
import torch, time, cProfile, pstats, sys
sys.path.insert(0,'.')
from zbot_lab_amd.envs import ZbotDirectEnvCfgV2, ZbotDirectEnvV2
cfg=ZbotDirectEnvCfgV2(); cfg.scene.num_envs=64
env=ZbotDirectEnvV2(cfg); env.reset()
a=torch.randn(64,6,device='cuda')
for k in range(100): env.step(a)
torch.cuda.synchronize()
pr=cProfile.Profile(); pr.enable()
for k in range(2000): env.step(a)
pr.disable(); torch.cuda.synchronize()
pstats.Stats(pr).sort_stats('tottime').print_stats(14)
" 2>&1 | tail -30
