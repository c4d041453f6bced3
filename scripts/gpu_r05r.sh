#!/bin/bash
# Round 5: the solve graph's mid-graph stalls (~250 us per solve in the kernel
# trace): A/B of one graph for factorisation + solve and of uploading the graphs
# after instantiation, on the headline step (3 timed steps each).
O=gpurun_out
for v in base PGO_ONE_GRAPH=1 PGO_GRAPH_UPLOAD=1 "PGO_ONE_GRAPH=1 PGO_GRAPH_UPLOAD=1"; do
  tag=$(echo $v | tr ' =' '__')
  if [ "$v" = base ]; then envs=""; else envs="$v"; fi
  env $envs timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --live 0 --gicp 0 --search 0 --marginals 0 --c5 0 --gn 0 --converged 0 --profile-every 0 > $O/r05r_$tag.json 2> $O/r05r_$tag.err || { echo "bench $v failed"; tail -3 $O/r05r_$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/r05r_$tag.json').read().strip().splitlines()[-1]); print('$v', round(d['value'],2), round(d['ms_per_step'],2), d['per_step']['final_error'])"
done
echo done
