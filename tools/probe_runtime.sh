set -o pipefail
echo "== torch imported first"
timeout -k 5 120 python -c "
import torch; torch.cuda.set_device(0); x=torch.zeros(1,device='cuda')
from narwhal_amd import _lib; e=_lib.Engine(device=0); print('torch-first ok', e.sha512(b'')[:4].hex(), torch.ones(2,device='cuda').sum().item())
" 2>&1 | tail -3
echo "== lib loaded first, torch init first"
timeout -k 5 120 python -c "
from narwhal_amd import _lib
import torch; torch.cuda.set_device(0); x=torch.zeros(1,device='cuda')
try:
    e=_lib.Engine(device=0); print('lib-loaded-first/torch-init-first ok')
except Exception as ex: print('FAIL', ex)
" 2>&1 | tail -3
echo "== lib loaded+init first, then torch"
timeout -k 5 120 python -c "
from narwhal_amd import _lib
e=_lib.Engine(device=0)
import torch
try:
    torch.cuda.set_device(0); x=torch.zeros(1,device='cuda'); print('lib-first ok')
except Exception as ex: print('FAIL', ex)
" 2>&1 | tail -3
exit 0
