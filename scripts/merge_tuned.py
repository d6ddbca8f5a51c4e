"""Merge TunableOp result tables: validator lines from the first file, entries from all (later wins).

    python scripts/merge_tuned.py OUT IN1 [IN2 ...]
"""
import sys


def main():
    out, ins = sys.argv[1], sys.argv[2:]
    validators, entries = [], {}
    for i, path in enumerate(ins):
        for line in open(path):
            line = line.strip()
            if not line:
                continue
            parts = line.split(",")
            if parts[0] == "Validator":
                if i == 0:
                    validators.append(line)
            else:
                entries[(parts[0], parts[1])] = line
    with open(out, "w") as f:
        f.write("\n".join(validators + list(entries.values())) + "\n")
    print(f"{out}: {len(entries)} entries")


if __name__ == "__main__":
    main()
