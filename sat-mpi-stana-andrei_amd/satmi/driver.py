"""The comparison / report driver of the reference, on the GPU solvers.

Same entry points, prompts, result strings and report format as REF.py; the
solvers behind the menu are satmi.solvers (libsatmi.so on the MI355X).

    read_formula_from_input()                      REF.py:33-59
    run_solver_with_timeout(func, formula, queue)  REF.py:408-414
    execute_with_timeout(func, formula, timeout)   REF.py:417-437
    save_results_to_file(formula, results, name)   REF.py:441-487
    main_menu()                                    REF.py:491-632

REF.py isolates every solver in a child process and terminates it at the
deadline.  A process that has initialised HIP cannot hand the GPU to a forked
child, so here the deadline travels into the solver instead: the DPLL kernel
checks it against the device clock, resolution and Davis-Putnam between passes
and steps, and an expired call returns the reference's "Timeout after N
seconds" message.  (The reference's parent also joins the child before it
drains the result queue, so there a result larger than a pipe buffer reads as
a timeout; here the result is returned.)
"""
import time
import tracemalloc

from . import solvers
from .dp import DavisPutnamLimit
from .resolution import ResolutionLimit
from .solvers import (SolverTimeout, cdcl_solve, davis_putnam_solver, dpll_optimized, generate_large_formula,
                      hybrid_solver, pysat_solver, resolution_solver)

TIMEOUT_SECONDS = 60
_DEADLINE_ERRORS = (SolverTimeout, ResolutionLimit, DavisPutnamLimit)


SOLVERS = {
    "1": ("Resolution", resolution_solver),
    "2": ("Davis-Putnam", davis_putnam_solver),
    "3": ("DPLL", dpll_optimized),
    "4": ("CDCL", cdcl_solve),
    "5": ("PySAT", pysat_solver),
    "6": ("Hybrid", hybrid_solver),
}


def read_formula_from_input(input_fn=input, print_fn=print):
    """Clauses typed one per line, DIMACS-style, 'done' to finish (REF.py:33-59)."""
    print_fn("\nEnter clauses one by line. End each clause with 0.")
    print_fn("Example: 1 -2 3 0 (this means x1 ∨ ¬x2 ∨ x3)")
    formula = []
    while True:
        while True:
            text = input_fn("Enter clause (or 'done' to finish): ").strip()
            if text.lower() == "done":
                return formula
            try:
                numbers = [int(tok) for tok in text.split()]
                if not numbers or numbers[-1] != 0:
                    print_fn("Error: Clause must end with 0")
                    continue
                clause = numbers[:-1]
                if any(x == 0 for x in clause):
                    print_fn("Error: 0 can only appear at end of clause")
                    continue
                formula.append(clause)
                break
            except ValueError:
                print_fn("Error: Please enter integers only")
        print_fn(f"Current formula: {len(formula)} clauses")


def run_solver_with_timeout(solver_func, formula, queue):
    """REF.py:408-414: the solver's outcome as ('result', value) or ('error', message)."""
    try:
        queue.put(("result", solver_func(formula)))
    except Exception as e:  # noqa: BLE001 - the reference reports every failure the same way
        queue.put(("error", str(e)))


def execute_with_timeout(solver_func, formula, timeout):
    """(result, None) or (None, message); an expired deadline gives the reference's
    'Timeout after N seconds' (REF.py:417-437)."""
    solvers.set_time_limit(timeout)
    try:
        return solver_func(formula), None
    except _DEADLINE_ERRORS:
        return None, f"Timeout after {timeout} seconds"
    except Exception as e:  # noqa: BLE001
        return None, str(e)
    finally:
        solvers.set_time_limit(0)


def describe_result(name, result):
    """The 'Result' text of one solver (REF.py:591-601)."""
    if name in ("Resolution", "Davis-Putnam"):
        return f"Formula is {'satisfiable' if result else 'unsatisfiable'}"
    if name == "CDCL":
        sat, assignment = result
        text = f"Formula is {'satisfiable' if sat else 'unsatisfiable'}"
        if sat:
            text += f"\nAssignment sample: {dict(list(assignment.items())[:5])}..."
        return text
    text = f"Found {len(result)} solution(s)" if result else "No solutions found"
    if result:
        text += f"\nFirst assignment sample: {dict(list(result[0].items())[:5])}..."
    return text


def run_solvers(formula, to_run, timeout=TIMEOUT_SECONDS, print_fn=print):
    """Run (name, solver) pairs on the formula, timing each and tracing the host
    heap like REF.py:567-620; returns the results dict save_results_to_file takes."""
    results = {}
    for name, solver in to_run:
        print_fn(f"\nRunning {name}...")
        tracemalloc.start()
        start = time.time()
        try:
            result, error = execute_with_timeout(solver, list(formula), timeout)
            end = time.time()
            _, peak = tracemalloc.get_traced_memory()
            tracemalloc.stop()
            if error:
                results[name] = {"time": timeout if "Timeout" in error else -1,
                                 "memory": peak / 1024 if peak >= 0 else -1, "output": error}
                print_fn(error)
                continue
            output = describe_result(name, result)
            results[name] = {"time": end - start, "memory": peak / 1024, "output": output}
            print_fn(output)
            print_fn(f"Time: {end - start:.6f} seconds")
            print_fn(f"Peak memory: {peak / 1024:.2f} KB")
        except Exception as e:  # noqa: BLE001
            tracemalloc.stop()
            print_fn(f"Error in {name}: {str(e)}")
            results[name] = {"time": -1, "memory": -1, "output": f"Error: {str(e)}"}
    return results


def _report_lines(formula, results):
    variables = {abs(lit) for clause in formula for lit in clause}
    row = "{:<15} {:<12} {:<15} {:<30}\n"
    out = ["\n" + "=" * 80 + "\n", "SAT SOLVER COMPARISON RESULTS\n",
           f"Generated at: {time.strftime('%Y-%m-%d %H:%M:%S')}\n", "\nFORMULA STATISTICS:\n",
           f"- Clauses: {len(formula)}\n", f"- Variables: {len(variables)}\n",
           f"- Avg clause length: {sum(len(c) for c in formula) / max(len(formula), 1):.2f}\n",
           "\nSOLVER PERFORMANCE:\n", row.format("Solver", "Time (s)", "Memory (KB)", "Result"), "-" * 80 + "\n"]
    for name, res in results.items():
        shown = res["output"] if len(res["output"]) <= 50 else res["output"][:50] + "..."
        out.append(row.format(name, f"{res['time']:.6f}" if res["time"] >= 0 else "Error",
                              f"{res['memory']:.2f}" if res["memory"] >= 0 else "Error", shown))
    out.append("\nTIMING COMPARISON:\n")
    timed = [(name, res["time"]) for name, res in results.items() if res["time"] >= 0]
    if timed:
        fastest = min(timed, key=lambda x: x[1])
        slowest = max(timed, key=lambda x: x[1])
        out.append(f"- Fastest solver: {fastest[0]} ({fastest[1]:.6f}s)\n")
        out.append(f"- Slowest solver: {slowest[0]} ({slowest[1]:.6f}s)\n")
        if len(timed) > 1:
            out.append(f"- Speed difference: {slowest[1] / fastest[1]:.2f}x\n")
    out.append("=" * 80 + "\n")
    return out


def save_results_to_file(formula, results, filename="results.txt", print_fn=print):
    """Append the comparison report to `filename` in the reference's format (REF.py:441-487)."""
    try:
        with open(filename, "a") as fh:
            fh.writelines(_report_lines(formula, results))
        print_fn(f"\nResults saved to {filename} (without clause details)")
    except IOError as e:
        print_fn(f"Error saving file: {e}")


def main_menu(input_fn=input, print_fn=print, solver_table=None, report_file="rezultat.txt"):
    """The interactive comparison tool (REF.py:491-632)."""
    table = SOLVERS if solver_table is None else solver_table
    print_fn("SAT Solver Comparison Tool")
    print_fn("=" * 40)
    print_fn(f"Note: All solvers will timeout after {TIMEOUT_SECONDS} seconds")
    while True:
        print_fn("\nMain Menu:")
        print_fn("1. Enter formula manually")
        print_fn("2. Generate random formula")
        print_fn("3. Exit")
        choice = input_fn("Choose option: ").strip()
        if choice == "3":
            print_fn("Exiting program.")
            return
        if choice == "1":
            formula = read_formula_from_input(input_fn, print_fn)
        elif choice == "2":
            try:
                num_clauses = int(input_fn("Number of clauses: "))
                max_literals = int(input_fn("Max literals per clause: "))
                num_vars = int(input_fn("Number of variables: "))
                formula = generate_large_formula(num_clauses, max_literals, num_vars)
                print_fn(f"Generated formula with {len(formula)} clauses")
                print_fn("\nSample of generated clauses:")
                for clause in formula[:5]:
                    print_fn(" ".join(map(str, clause)) + " 0")
                if len(formula) > 5:
                    print_fn(f"... and {len(formula) - 5} more clauses")
            except ValueError:
                print_fn("Invalid input! Please enter integers.")
                continue
        else:
            print_fn("Invalid choice")
            continue
        variables = {abs(lit) for clause in formula for lit in clause}
        print_fn("\nFormula statistics:")
        print_fn(f"- Clauses: {len(formula)}")
        print_fn(f"- Variables: {len(variables)}")
        print_fn(f"- Avg clause length: {sum(len(c) for c in formula) / max(len(formula), 1):.2f}")
        print_fn("\nSelect solvers to compare:")
        for key, (name, _) in table.items():
            print_fn(f"{key}. {name}")
        print_fn("7. All solvers")
        print_fn("8. Back to main menu")
        while True:
            picked = input_fn("\nEnter choices (comma separated, or 7 for all): ").strip()
            if picked == "8":
                break
            keys = picked.split(",")
            to_run = list(table.values()) if "7" in keys else [table[k] for k in keys if k in table]
            if not to_run:
                print_fn("No valid solvers selected")
                continue
            results = run_solvers(formula, to_run, TIMEOUT_SECONDS, print_fn)
            if input_fn("\nSave these results to file? (y/n): ").lower() == "y":
                save_results_to_file(formula, results, report_file, print_fn)
            print_fn("\n1. Run more solvers on same formula")
            print_fn("2. Back to main menu")
            if input_fn("Choose option: ").strip() == "2":
                break


if __name__ == "__main__":
    main_menu()
