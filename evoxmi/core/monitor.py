"""Monitor base class (reference ``src/evox/core/monitor.py:1-47``).

Monitors live outside the state tree.  ``hooks()`` names the callbacks the
workflow must call; the workflow fires them in the order
``pre_step, pre_ask, post_ask, pre_eval, post_eval, pre_tell, post_tell, post_step``.
"""


class Monitor:
    def __init__(self):
        pass

    def set_opt_direction(self, opt_direction):
        pass

    def hooks(self):
        raise NotImplementedError

    def pre_step(self, state):
        pass

    def pre_ask(self, state):
        pass

    def post_ask(self, state, cand_sol):
        pass

    def pre_eval(self, state, cand_sol, transformed_cand_sol):
        pass

    def post_eval(self, state, cand_sol, transformed_cand_sol, fitness):
        pass

    def pre_tell(self, state, cand_sol, transformed_cand_sol, fitness, transformed_fitness):
        pass

    def post_tell(self, state):
        pass

    def post_step(self, state):
        pass
