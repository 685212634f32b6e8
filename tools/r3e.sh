for w in 4 1; do
timeout -k 5 30 ./tools/micro/chain_role 0 $w
timeout -k 5 30 ./tools/micro/chain_role_noslow 1 $w
timeout -k 5 30 ./tools/micro/chain_role_noslow 2 $w
done
