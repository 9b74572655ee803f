"""``LinProg`` -- the reference's modelling front-end is an empty stub
(``lpsol/linprog.py:383-393``) that nothing connects to Tableau/Simplex
(SURVEY.md §2, §3.4).  It is kept importable with the same (empty)
behaviour; LinExpr/LinCon/LinVar are outside the pivot hot path and are not
rebuilt here."""


class LinProg:
    '''
    representation of a linear program in possibly non standard form
    (empty in the reference)
    '''

    def __init__(self):
        '''
        '''
