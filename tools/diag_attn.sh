set -o pipefail
export TMPDIR=/tmp
python -c "import torch; p=torch.cuda.get_device_properties(0); print(p.multi_processor_count, p.name)"
timeout -k 10 200 python -u tools/attn_bench.py 21 197 12 64 0 42 197 12 64 0 84 197 12 64 0 256 197 12 64 0
timeout -k 10 200 python -u abase/tools/attn_bench.py 21 197 12 64 0 42 197 12 64 0 84 197 12 64 0 256 197 12 64 0
