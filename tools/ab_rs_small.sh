set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 1 0 1 0; do
  DCC_RS_SMALL=$v timeout -k 10 200 python3 bench.py --only C4,MAAT_C2,MAAT_1M --steps 8 --warmup 2 2>/dev/null | python3 -c "import json,sys;j=json.load(sys.stdin);print('small=$v',{k:round(v['device_ms'],3) for k,v in j.items()})" || exit 1
done
