# Source-able helper: load_env_file FILE
# Exports the KEY=VALUE lines of FILE without evaluating them as shell code
# (values with spaces, '$' or quotes are taken literally; one pair of matching
# surrounding quotes is stripped).  Variables already set in the environment win,
# so `VAR=x ./run-*.sh` overrides the file.  Comments and blank lines are skipped.
load_env_file() {
  local file="$1" line key val
  [ -f "$file" ] || return 0
  while IFS= read -r line || [ -n "$line" ]; do
    line="${line%$'\r'}"
    case "$line" in ''|'#'*) continue ;; esac
    line="${line#export }"
    key="${line%%=*}"
    [ "$key" = "$line" ] && continue            # no '='
    key="${key//[[:space:]]/}"
    [[ "$key" =~ ^[A-Za-z_][A-Za-z0-9_]*$ ]] || continue
    val="${line#*=}"
    if [[ ${#val} -ge 2 && ( ( "${val:0:1}" == '"' && "${val: -1}" == '"' ) || \
                             ( "${val:0:1}" == "'" && "${val: -1}" == "'" ) ) ]]; then
      val="${val:1:${#val}-2}"
    fi
    if [ -z "${!key+x}" ]; then
      export "$key=$val"
    fi
  done < "$file"
}
