cd $GRAFT_REPO_ROOT
for n in 51 102 204; do for k in d s; do arg=""; [ $k == s ] && arg=s; timeout -k 5 60 ./scripts/kbench $n r q $arg | grep full | sed "s/^/n=$n /"; done; done
